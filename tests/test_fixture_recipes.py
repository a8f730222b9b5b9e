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
    """forward_ref_bench.npz stores no inputs: every 4th protein of bench.py's workload (and every
    16th of config 5's) must regenerate to the SHA-256 the reference forward ran on."""
    FB = refwide.load_bench()
    assert refwide.cases(FB, "bench256_") == sorted(f"bench256_p{p}" for p in range(0, 1024, 4))
    # config 5's sample (make_forward_bench.py --config 5): every 16th of 512 x 512 residues
    assert refwide.cases(FB, "bench512_") == sorted(f"bench512_p{p}" for p in range(0, 512, 16))
    names = refwide.cases(FB)
    for c in names:
        n_res, seed = (int(v) for v in FB[c + "/synthetic_args"])
        assert (n_res, seed) == (int(c[5:8]), 1000 + int(c.split("_p")[1]))
        s = synthetic.synthetic_protein(n_res, seed)
        assert M.input_sha(s.atom37_positions.astype(np.float32), s.atom_flags()) == str(FB[c + "/input_sha256"]), c
