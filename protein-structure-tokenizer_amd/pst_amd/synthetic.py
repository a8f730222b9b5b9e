"""Synthetic backbone generator for benchmarks and parity tests.

Protein p uses `numpy.random.default_rng(seed + p)`. CA atoms follow a persistent random walk
with 3.8 Å steps (bond angle ≈ 90–125°), N/C/O are placed from the local frame with ideal-ish
geometry (non-collinear N-CA-C), residues are ALA with gt atoms {N, CA, C, O} (CB absent).
Coordinates are rounded to 3 decimals (as in PDB text) then to float32, and stored in float64 —
exactly the representation the PDB path produces, so residue centroids are exact in float64.
"""
import hashlib
import math
from typing import List

import numpy as np

from . import residue_constants as rc
from .sample import ProteinStructureSample


def _unit(x, y, z):
    n = math.sqrt(x * x + y * y + z * z)
    return x / n, y / n, z / n


def synthetic_protein(n_res: int, seed: int) -> ProteinStructureSample:
    rng = np.random.default_rng(seed)
    noise = rng.normal(size=(n_res, 64, 3)).tolist()  # rejection-sampling pool per step
    jit = (1e-3 * rng.normal(size=(n_res, 2, 3))).tolist()
    ca = [(0.0, 0.0, 0.0)]
    d = _unit(*rng.normal(size=3).tolist())
    for i in range(1, n_res):
        pool = noise[i]
        for c in range(64):
            e = pool[c]
            cand = _unit(d[0] + 1.1 * e[0], d[1] + 1.1 * e[1], d[2] + 1.1 * e[2])
            cosang = cand[0] * d[0] + cand[1] * d[1] + cand[2] * d[2]
            if -0.55 < cosang < 0.35:  # turn of ~70-123 degrees between successive steps
                break
        d = cand
        p = ca[-1]
        ca.append((p[0] + 3.8 * d[0], p[1] + 3.8 * d[1], p[2] + 3.8 * d[2]))
    pos = np.zeros((n_res, rc.atom_type_num, 3))
    for i in range(n_res):
        c0 = ca[i]
        pv = ca[i] if i > 0 else ca[1]
        pm = ca[i - 1] if i > 0 else ca[0]
        prev_d = (pv[0] - pm[0], pv[1] - pm[1], pv[2] - pm[2])
        if i + 1 < n_res:
            nx = ca[i + 1]
            next_d = (nx[0] - c0[0], nx[1] - c0[1], nx[2] - c0[2])
        else:
            next_d = prev_d
        j0, j1 = jit[i]
        b = _unit(prev_d[0] - next_d[0] + j0[0], prev_d[1] - next_d[1] + j0[1], prev_d[2] - next_d[2] + j0[2])
        cr = (prev_d[1] * next_d[2] - prev_d[2] * next_d[1], prev_d[2] * next_d[0] - prev_d[0] * next_d[2],
              prev_d[0] * next_d[1] - prev_d[1] * next_d[0])
        nrm = _unit(cr[0] + j1[0], cr[1] + j1[1], cr[2] + j1[2])
        nd = _unit(*next_d)
        N = _unit(0.55 * b[0] - 0.8 * nd[0] + 0.2 * nrm[0], 0.55 * b[1] - 0.8 * nd[1] + 0.2 * nrm[1],
                  0.55 * b[2] - 0.8 * nd[2] + 0.2 * nrm[2])
        C = _unit(0.55 * b[0] + 0.8 * nd[0] - 0.2 * nrm[0], 0.55 * b[1] + 0.8 * nd[1] - 0.2 * nrm[1],
                  0.55 * b[2] + 0.8 * nd[2] - 0.2 * nrm[2])
        O = _unit(b[0] + 0.3 * nrm[0], b[1] + 0.3 * nrm[1], b[2] + 0.3 * nrm[2])
        pos[i, rc.CA_INDEX] = c0
        pos[i, rc.N_INDEX] = (c0[0] + 1.46 * N[0], c0[1] + 1.46 * N[1], c0[2] + 1.46 * N[2])
        cc = (c0[0] + 1.52 * C[0], c0[1] + 1.52 * C[1], c0[2] + 1.52 * C[2])
        pos[i, rc.C_INDEX] = cc
        pos[i, rc.O_INDEX] = (cc[0] + 1.23 * O[0], cc[1] + 1.23 * O[1], cc[2] + 1.23 * O[2])
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
