"""`ProteinStructureSample` data contract (mirror of
`structure_tokenizer/data/protein_structure_sample.py:27-70`)."""
from typing import NamedTuple, Optional

import numpy as np

from . import residue_constants as rc


class ProteinStructureSample(NamedTuple):
    chain_id: Optional[str]
    nb_residues: int
    aatype: np.ndarray  # [n, 21] one-hot
    atom37_positions: np.ndarray  # [n, 37, 3] float64 holding float32-exact values (PDB path)
    atom37_gt_exists: np.ndarray  # [n, 37] bool
    atom37_atom_exists: np.ndarray  # [n, 37] bool
    resolution: float
    pdb_cluster_size: int

    def get_missing_backbone_coords_mask(self) -> np.ndarray:
        """True where N, CA, C or O is missing (`protein_structure_sample.py:64-70`)."""
        g = self.atom37_gt_exists
        return ~(g[:, rc.CA_INDEX] & g[:, rc.N_INDEX] & g[:, rc.C_INDEX] & g[:, rc.O_INDEX])

    def atom_flags(self) -> np.ndarray:
        """Packed per-atom flags handed to the device: bit0 = gt_exists, bit1 = atom_exists."""
        return (self.atom37_gt_exists.astype(np.uint8)
                | (self.atom37_atom_exists.astype(np.uint8) << 1))


def sample_from_arrays(positions: np.ndarray, flags: np.ndarray, aatype_idx=None) -> ProteinStructureSample:
    """Inverse of `atom_flags`: a sample from atom37 positions + packed flags (aatype ALA unless
    given as residue indices; the tokenize path never reads it)."""
    n = positions.shape[0]
    aa = np.zeros((n, rc.restype_num + 1))
    idx = np.full(n, rc.restype_order["A"]) if aatype_idx is None else np.asarray(aatype_idx)
    aa[np.arange(n), idx] = 1.0
    return ProteinStructureSample(None, n, aa, np.asarray(positions, dtype=np.float64),
                                  (flags & 1).astype(bool), (flags & 2).astype(bool), 0.0, 1)
