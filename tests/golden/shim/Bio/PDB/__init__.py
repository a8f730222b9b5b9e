class PDBParser:  # import-only stub; fixtures bypass PDB text parsing
    def __init__(self, *a, **k):
        raise NotImplementedError("Biopython is not available in this container")
