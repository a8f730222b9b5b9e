"""Synthetic backbone generator for benchmarks and parity tests.

Protein p uses `numpy.random.default_rng(seed + p)`. CA atoms follow a persistent random walk
with 3.8 Å steps (bond angle ≈ 90–125°), N/C/O are placed from the local frame with ideal-ish
geometry (non-collinear N-CA-C), residues are ALA with gt atoms {N, CA, C, O} (CB absent).
Coordinates are rounded to 3 decimals (as in PDB text) then to float32, and stored in float64 —
exactly the representation the PDB path produces, so residue centroids are exact in float64.
"""
import hashlib
from typing import List

import numpy as np

from . import residue_constants as rc
from .sample import ProteinStructureSample


def _unit(v):
    return v / np.linalg.norm(v)


def synthetic_protein(n_res: int, seed: int) -> ProteinStructureSample:
    rng = np.random.default_rng(seed)
    ca = np.zeros((n_res, 3))
    d = _unit(rng.normal(size=3))
    for i in range(1, n_res):
        while True:
            cand = _unit(d + rng.normal(scale=1.1, size=3))
            cosang = float(np.dot(cand, d))
            if -0.55 < cosang < 0.35:  # turn of ~70–123 degrees between successive steps
                break
        d = cand
        ca[i] = ca[i - 1] + 3.8 * d
    pos = np.zeros((n_res, rc.atom_type_num, 3))
    for i in range(n_res):
        prev_d = ca[i] - ca[i - 1] if i > 0 else ca[1] - ca[0]
        next_d = ca[i + 1] - ca[i] if i + 1 < n_res else prev_d
        b = _unit(prev_d - next_d + 1e-3 * rng.normal(size=3))
        nrm = _unit(np.cross(prev_d, next_d) + 1e-3 * rng.normal(size=3))
        pos[i, rc.CA_INDEX] = ca[i]
        pos[i, rc.N_INDEX] = ca[i] + 1.46 * _unit(0.55 * b - 0.8 * _unit(next_d) + 0.2 * nrm)
        pos[i, rc.C_INDEX] = ca[i] + 1.52 * _unit(0.55 * b + 0.8 * _unit(next_d) - 0.2 * nrm)
        pos[i, rc.O_INDEX] = pos[i, rc.C_INDEX] + 1.23 * _unit(b + 0.3 * nrm)
    pos = np.round(pos, 3).astype(np.float32).astype(np.float64)
    gt = np.zeros((n_res, rc.atom_type_num), dtype=bool)
    gt[:, [rc.N_INDEX, rc.CA_INDEX, rc.C_INDEX, rc.O_INDEX]] = True
    exists = np.tile(np.asarray(rc.res_atom37_exist["ALA"], dtype=bool), (n_res, 1))
    aatype = np.zeros((n_res, rc.restype_num + 1))
    aatype[:, rc.restype_order["A"]] = 1.0
    pos[~gt] = 0.0
    return ProteinStructureSample(None, n_res, aatype, pos, gt, exists, 0.0, 1)


def synthetic_batch(n_prot: int, n_res: int, seed: int = 1000) -> List[ProteinStructureSample]:
    return [synthetic_protein(n_res, seed + p) for p in range(n_prot)]


def batch_sha256(samples: List[ProteinStructureSample]) -> str:
    h = hashlib.sha256()
    for s in samples:
        h.update(s.atom37_positions.tobytes())
        h.update(s.atom37_gt_exists.tobytes())
    return h.hexdigest()
