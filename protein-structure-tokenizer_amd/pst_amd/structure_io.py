"""atom37 structure → PDB text, in the reference's writer format (`structure_tokenizer/data/
protein.py:192-296`, `Protein.from_atom37_rep` :86-111): MODEL 1, one ATOM line per present
atom, 0-based residue numbers, occupancy 1.00, B-factor 0.00, TER, ENDMDL, END, lines padded to 80.
"""
import numpy as np

from . import residue_constants as rc

PDB_CHAIN_IDS = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789"


def _res3(a: int) -> str:
    restypes = rc.restypes + ["X"]
    return rc.restype_1to3.get(restypes[a], "UNK")


def atom37_to_pdb(atom37_positions: np.ndarray, atom37_mask: np.ndarray, aatype: np.ndarray,
                  chain_id: str = "A") -> str:
    """`to_pdb(Protein.from_atom37_rep(positions, mask, mask, one_hot(aatype), chain_id))`."""
    if chain_id not in PDB_CHAIN_IDS:
        raise ValueError(f"invalid chain id {chain_id!r}")
    aatype = np.asarray(aatype).astype(np.int64)
    if np.any(aatype > rc.restype_num):
        raise ValueError("Invalid aatypes.")
    lines = ["MODEL     1"]
    atom_index = 1
    n = aatype.shape[0]
    for i in range(n):
        res3 = _res3(int(aatype[i]))
        for atom_name, pos, m in zip(rc.atom_types, atom37_positions[i], atom37_mask[i]):
            if m < 0.5:
                continue
            name = atom_name if len(atom_name) == 4 else f" {atom_name}"
            lines.append(f"{'ATOM':<6}{atom_index:>5} {name:<4}{'':>1}{res3:>3} {chain_id:>1}{i:>4}{'':>1}   "
                         f"{pos[0]:>8.3f}{pos[1]:>8.3f}{pos[2]:>8.3f}{1.0:>6.2f}{0.0:>6.2f}          "
                         f"{atom_name[0]:>2}{'':>2}")
            atom_index += 1
    last = _res3(int(aatype[-1])) if n else "UNK"
    lines.append(f"{'TER':<6}{atom_index:>5}      {last:>3} {chain_id:>1}{max(n - 1, 0):>4}")
    lines.append("ENDMDL")
    lines.append("END")
    return "\n".join(line.ljust(80) for line in lines) + "\n"
