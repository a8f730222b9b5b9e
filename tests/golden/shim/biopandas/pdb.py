class PandasPdb:  # import-only stub (get_CA_coords is off the tokenize path)
    def read_pdb(self, *a, **k):
        raise NotImplementedError("biopandas is not available")
