"""Fixture recipes cannot drift from the committed data: the synthetic inputs of
`forward_ref_wide.npz` are regenerated with today's `pst_amd.synthetic` and must hash to the
SHA-256 stored beside them; the other fixtures' generators read their stored inputs back
(`make_golden.py forward` reuses `forward_golden_f64.npz`'s inputs when the file exists)."""
import numpy as np

import make_forward_wide as M
import refwide
from pst_amd import synthetic

F = refwide.load()


def test_wide_synthetic_inputs_reproduce():
    checked = 0
    for c in refwide.cases(F):
        if c + "/input_sha256" not in F.files:
            continue
        n_res, seed = (int(v) for v in F[c + "/synthetic_args"])
        s = synthetic.synthetic_protein(n_res, seed)
        pos, fl = s.atom37_positions.astype(np.float32), s.atom_flags()
        assert M.input_sha(pos, fl) == str(F[c + "/input_sha256"]), c
        assert np.array_equal(pos, F[c + "/in_positions"]) and np.array_equal(fl, F[c + "/in_flags"])
        checked += 1
    assert checked == 14  # bench256 p0-7, p200, p511, p777, p1023; bench512 p0-1


def test_bench_workload_is_the_fixture_workload():
    """bench.py's proteins p (seed 1000 + p, 256 residues) are the fixture's bench256 cases, in its
    first pipeline chunk (0, 1) and in the later ones (200, 511, 777, 1023)."""
    for p in (0, 1, 200, 511, 777, 1023):
        s = synthetic.synthetic_protein(256, 1000 + p)
        assert np.array_equal(s.atom37_positions.astype(np.float32), F[f"bench256_p{p}_k4096_df1/in_positions"])


def test_casp14_inputs_match_atom37_fixture():
    C = np.load(M.os.path.join(M.HERE, "casp14_atom37.npz"))
    for i, nm in enumerate(C["names"]):
        a, b = int(C["offsets"][i]), int(C["offsets"][i + 1])
        for cb in (4096, 64000):
            assert np.array_equal(F[f"casp_{nm}_k{cb}_df1/in_positions"], C["positions"][a:b])


def test_bench_fixture_inputs_reproduce():
    """forward_ref_bench.npz stores no inputs: every protein of bench.py's headline workload (and
    of config 5's) must regenerate to the SHA-256 the reference forward ran on. The full-latent
    subset (compact_bench.FULL_EVERY / FULL_PHASE) agrees with the token ids and margins."""
    import compact_bench as CB
    for name, n_res, n_prot in (("bench256", 256, 1024), ("bench512", 512, 512)):
        S = refwide.load_bench_sample(name)
        prots = [int(p) for p in S.proteins]
        assert prots == list(range(n_prot))
        assert sorted(S.full) == [p for p in prots if p % CB.FULL_EVERY[name] == CB.FULL_PHASE[name]]
        for p, fb in S.full.items():
            i = S.index[p]
            m = S.margin[S.tok_off[i]:S.tok_off[i + 1]]
            assert fb.shape == (S.n_tokens(p), S.meta["D"])
            # float32-stored latents: their margins within float32 rounding of the stored ones
            assert np.abs(refwide.dim_margins(fb).min(-1) - m).max() < 1e-6, (name, p)
        assert S.meta["n_res"] == n_res and S.meta["seed0"] == 1000
        assert len(S.tok_off) == len(prots) + 1 and S.tok_off[-1] == len(S.tokens) == len(S.margin)
        assert (S.margin[S.close] < refwide.CLOSE).all() and (np.delete(S.margin, S.close) >= refwide.CLOSE).all()
        assert np.array_equal(refwide.dim_margins(S.close_bounded).min(-1).astype(np.float32), S.margin[S.close])
        for i, p in enumerate(prots):
            s = synthetic.synthetic_protein(n_res, 1000 + p)
            assert M.input_sha(s.atom37_positions.astype(np.float32), s.atom_flags()) == str(S.input_sha256[i]), p
