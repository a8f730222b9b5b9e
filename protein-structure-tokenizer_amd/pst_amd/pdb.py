"""PDB text → `ProteinStructureSample` (restatement of the Biopython-based parser in
`structure_tokenizer/data/protein_structure_sample.py:166-248`).

Biopython is not part of this build, so the PDB fixed-column format is read directly with the
semantics `Bio.PDB.PDBParser(QUIET=True)` gives the reference:
  * records are named by their exact first 6 columns ("ATOM  ", "HETATM", "MODEL ", "ENDMDL");
    the header ends at the first ATOM/HETATM/MODEL record and coordinates end at the first
    "CONECT" or "END   " record (Bio's `_get_header` / `_parse_coordinates`);
  * only the first MODEL exists, or ValueError("Only single model PDBs ...") for >1 model;
  * ATOM and HETATM records both create residues (waters included), grouped per chain in order
    of first appearance, residues in file order, keyed by (het-flag, resseq, icode);
  * an insertion code raises ValueError (`:187-191`);
  * coordinates are float32 (Bio stores `atom.coord` as float32) held in float64 arrays;
  * alternate locations: the highest-occupancy altloc of an atom is kept (first on ties);
    a repeated atom name without altloc keeps the first record;
  * residue names outside the 20 standard types become UNK (aatype 20); atoms outside atom37
    are ignored; a residue with no atom37 atom is skipped (`:228-230`).
"""
from collections import OrderedDict
from typing import Optional

import numpy as np

from . import residue_constants as rc
from .sample import ProteinStructureSample


def _parse_records(pdb_str: str):
    models = 0
    seen_atom_before_model = False
    chains: "OrderedDict[str, OrderedDict]" = OrderedDict()
    in_first = True
    started = False  # Bio's header ends at the first "ATOM  " / "HETATM" / "MODEL " record
    for line in pdb_str.splitlines():
        rec = line[:6]  # Bio compares the 6-column record name exactly
        if not started:
            if rec not in ("ATOM  ", "HETATM", "MODEL "):
                continue
            started = True
        if rec in ("END   ", "CONECT"):
            break  # end of atomic data: Bio stops reading coordinates here
        if rec == "MODEL ":
            models += 1
            in_first = models == 1
            continue
        if rec == "ENDMDL":
            in_first = False
            continue
        if rec not in ("ATOM  ", "HETATM"):
            continue
        if models == 0:
            seen_atom_before_model = True
        if not in_first and models > 0:
            continue
        line = line.ljust(80)
        name = line[12:16].strip()
        altloc = line[16]
        resname = line[17:20].strip()
        chain = line[21]
        resseq = int(line[22:26])
        icode = line[26]
        x, y, z = float(line[30:38]), float(line[38:46]), float(line[46:54])
        occ_s = line[54:60].strip()
        occ = float(occ_s) if occ_s else 0.0
        if rec.startswith("HETATM"):
            het = "W" if resname in ("HOH", "WAT") else "H_" + resname
        else:
            het = " "
        res_key = (het, resseq, icode)
        residues = chains.setdefault(chain, OrderedDict())
        res = residues.get(res_key)
        if res is None:
            res = {"resname": resname, "icode": icode, "resseq": resseq, "atoms": OrderedDict()}
            residues[res_key] = res
        coord = np.array((x, y, z), dtype=np.float32)
        prev = res["atoms"].get(name)
        if prev is None:
            res["atoms"][name] = (coord, occ, altloc)
        elif altloc != " " and occ > prev[1]:
            res["atoms"][name] = (coord, occ, altloc)
    n_models = max(models, 1) if (models or seen_atom_before_model) else 0
    return n_models, chains


def protein_structure_from_pdb_string(pdb_str: str, chain_id: Optional[str] = None
                                      ) -> ProteinStructureSample:
    n_models, chains = _parse_records(pdb_str)
    if n_models != 1:
        raise ValueError(f"Only single model PDBs are supported. Found {n_models} models.")
    positions, aatype, masks, exists = [], [], [], []
    for cid, residues in chains.items():
        if chain_id is not None and cid != chain_id:
            continue
        for (het, resseq, icode), res in residues.items():
            if icode != " ":
                raise ValueError(
                    f"PDB contains an insertion code at chain {cid} and residue index "
                    f"{resseq}. These are not supported.")
            short = rc.restype_3to1.get(res["resname"], "X")
            res_name = rc.restype_1to3.get(short, "UNK")
            idx = rc.restype_order.get(short, rc.restype_num)
            pos = np.zeros((rc.atom_type_num, 3))
            mask = np.zeros((rc.atom_type_num,))
            for name, (coord, _, _) in res["atoms"].items():
                if name not in rc.atom_order:
                    continue
                pos[rc.atom_order[name]] = coord
                mask[rc.atom_order[name]] = 1.0
            if np.sum(mask) < 0.5:
                continue
            aatype.append(idx)
            positions.append(pos)
            masks.append(mask)
            exists.append(np.asarray(rc.res_atom37_exist[res_name]))
    n = len(positions)
    onehot = np.zeros((n, rc.restype_num + 1))
    if n:
        onehot[np.arange(n), np.asarray(aatype)] = 1.0
    return ProteinStructureSample(
        chain_id=chain_id,
        nb_residues=n,
        aatype=onehot,
        atom37_positions=np.asarray(positions).reshape(n, rc.atom_type_num, 3),
        atom37_gt_exists=np.asarray(masks).reshape(n, rc.atom_type_num).astype(bool),
        atom37_atom_exists=np.asarray(exists).reshape(n, rc.atom_type_num).astype(bool),
        resolution=0.0,
        pdb_cluster_size=1,
    )


def protein_structure_from_pdb_file(path: str) -> ProteinStructureSample:
    with open(path, "r") as fh:
        return protein_structure_from_pdb_string(fh.read())


def to_pdb_string(sample: ProteinStructureSample, chain_id: str = "A") -> str:
    """Minimal ATOM-record writer (the fields the parser above reads): one residue per row of
    `sample`, atoms present in `atom37_gt_exists`, coordinates %8.3f. Used to build PDB inputs
    for end-to-end CLI tests; the reference's full writer (`data/protein.py:to_pdb`) belongs to
    the decode path."""
    lines = []
    serial = 1
    aat = np.argmax(sample.aatype, axis=-1) if sample.aatype.size else np.zeros(sample.nb_residues, int)
    for i in range(sample.nb_residues):
        a = int(aat[i])
        resname = rc.restype_1to3.get(rc.restypes[a], "UNK") if a < rc.restype_num else "UNK"
        for j, name in enumerate(rc.atom_types):
            if not sample.atom37_gt_exists[i, j]:
                continue
            x, y, z = (float(v) for v in sample.atom37_positions[i, j])
            nm = name if len(name) == 4 else " " + name
            lines.append(f"ATOM  {serial:5d} {nm:<4s} {resname:>3s} {chain_id}{i + 1:4d}    "
                         f"{x:8.3f}{y:8.3f}{z:8.3f}{1.0:6.2f}{0.0:6.2f}          {name[0]:>2s}")
            serial += 1
    lines.append("END")
    return "\n".join(lines) + "\n"
