"""Residue/atom tables needed by the tokenize path (restated, AF2 conventions).

Mirrors the subset of `structure_tokenizer/data/residue_constants.py` that the PDB parser and
graph builder read: the atom37 ordering (`:539-579`), the 20-letter restype order (`:706-729`),
the 1<->3 letter maps (`:812-840`) and `res_atom37_exist` (`:733-737`, UNK = N, CA, C, CB).
`tests/test_reference_tables.py` checks every table against the reference module.
"""
from typing import Dict, List

atom_types: List[str] = [
    "N", "CA", "C", "CB", "O", "CG", "CG1", "CG2", "OG", "OG1", "SG", "CD", "CD1", "CD2",
    "ND1", "ND2", "OD1", "OD2", "SD", "CE", "CE1", "CE2", "CE3", "NE", "NE1", "NE2", "OE1",
    "OE2", "CH2", "NH1", "NH2", "OH", "CZ", "CZ2", "CZ3", "NZ", "OXT",
]
atom_order: Dict[str, int] = {a: i for i, a in enumerate(atom_types)}
atom_type_num = len(atom_types)  # 37
N_INDEX, CA_INDEX, C_INDEX, O_INDEX = (atom_order[a] for a in ("N", "CA", "C", "O"))

restypes: List[str] = list("ARNDCQEGHILKMFPSTWYV")
restype_order: Dict[str, int] = {r: i for i, r in enumerate(restypes)}
restype_num = len(restypes)  # 20; index 20 = UNK

restype_1to3: Dict[str, str] = {
    "A": "ALA", "R": "ARG", "N": "ASN", "D": "ASP", "C": "CYS", "Q": "GLN", "E": "GLU",
    "G": "GLY", "H": "HIS", "I": "ILE", "L": "LEU", "K": "LYS", "M": "MET", "F": "PHE",
    "P": "PRO", "S": "SER", "T": "THR", "W": "TRP", "Y": "TYR", "V": "VAL",
}
restype_3to1: Dict[str, str] = {v: k for k, v in restype_1to3.items()}

# Heavy atoms present in each standard residue (atom37 names).
residue_atoms: Dict[str, List[str]] = {
    "ALA": ["C", "CA", "CB", "N", "O"],
    "ARG": ["C", "CA", "CB", "CG", "CD", "CZ", "N", "NE", "O", "NH1", "NH2"],
    "ASP": ["C", "CA", "CB", "CG", "N", "O", "OD1", "OD2"],
    "ASN": ["C", "CA", "CB", "CG", "N", "ND2", "O", "OD1"],
    "CYS": ["C", "CA", "CB", "N", "O", "SG"],
    "GLU": ["C", "CA", "CB", "CG", "CD", "N", "O", "OE1", "OE2"],
    "GLN": ["C", "CA", "CB", "CG", "CD", "N", "NE2", "O", "OE1"],
    "GLY": ["C", "CA", "N", "O"],
    "HIS": ["C", "CA", "CB", "CG", "CD2", "CE1", "N", "ND1", "NE2", "O"],
    "ILE": ["C", "CA", "CB", "CG1", "CG2", "CD1", "N", "O"],
    "LEU": ["C", "CA", "CB", "CG", "CD1", "CD2", "N", "O"],
    "LYS": ["C", "CA", "CB", "CG", "CD", "CE", "N", "NZ", "O"],
    "MET": ["C", "CA", "CB", "CG", "CE", "N", "O", "SD"],
    "PHE": ["C", "CA", "CB", "CG", "CD1", "CD2", "CE1", "CE2", "CZ", "N", "O"],
    "PRO": ["C", "CA", "CB", "CG", "CD", "N", "O"],
    "SER": ["C", "CA", "CB", "N", "O", "OG"],
    "THR": ["C", "CA", "CB", "CG2", "N", "O", "OG1"],
    "TRP": ["C", "CA", "CB", "CG", "CD1", "CD2", "CE2", "CE3", "CZ2", "CZ3", "CH2", "N",
            "NE1", "O"],
    "TYR": ["C", "CA", "CB", "CG", "CD1", "CD2", "CE1", "CE2", "CZ", "N", "O", "OH"],
    "VAL": ["C", "CA", "CB", "CG1", "CG2", "N", "O"],
}
res_atom37_exist: Dict[str, List[float]] = {
    r: [float(a in atoms) for a in atom_types] for r, atoms in residue_atoms.items()
}
res_atom37_exist["UNK"] = [1.0, 1.0, 1.0, 1.0] + 33 * [0.0]
