"""N>1 path on CPU: two gloo ranks (127.0.0.1), each takes GPU LOCAL_RANK's LPT shard of the PDB
list through the CLI; the union of their token files must equal a single-process run. Plus the
cross-rank codebook perplexity (the one collective: an all-reduce of K float64)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from pst_amd import params as P
from pst_amd import pdb, synthetic
from test_host import OracleTokenizeFn  # noqa: F401  (imported by the worker too)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_rank_cli_sharding(tmp_path):
    import _mr_worker
    pdb_dir = tmp_path / "pdbs"
    pdb_dir.mkdir()
    ss = {f"p{i}": synthetic.synthetic_protein(50 + 3 * i, 70 + i) for i in range(5)}
    for k, s in ss.items():
        (pdb_dir / f"{k}.pdb").write_text(pdb.to_pdb_string(s))
    mdir = tmp_path / "model"
    mdir.mkdir()
    P.save_params_npz(str(mdir / "params.npz"), P.random_full_params(6, seed=21))
    out = tmp_path / "tok"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mr_worker.run, args=(r, 2, port, str(pdb_dir), str(mdir), str(out), q))
             for r in range(2)]
    for p in procs:
        p.start()
    shards = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(sum(shards, [])) == sorted(f"{k}.pdb" for k in ss)
    assert not set(shards[0]) & set(shards[1])
    assert sorted(os.listdir(out)) == sorted(f"{k}_tokens.npy" for k in ss)
    from oracle import oracle as O
    blob = P.pack(P.random_full_params(6, seed=21), 6)
    for k, s in ss.items():
        t = np.load(out / f"{k}_tokens.npy")
        want = O.tokenize(blob, (4,) * 6, 1, s.atom37_positions, s.atom_flags())["tokens"]
        assert np.array_equal(t[0], want)


def test_two_rank_cli_existing_output_dir(tmp_path):
    """Rank 0 creates --token_save_path with exist_ok=False; if it exists, every rank raises."""
    import _mr_worker
    pdb_dir = tmp_path / "pdbs"
    pdb_dir.mkdir()
    (pdb_dir / "p0.pdb").write_text(pdb.to_pdb_string(synthetic.synthetic_protein(55, 3)))
    mdir = tmp_path / "model"
    mdir.mkdir()
    P.save_params_npz(str(mdir / "params.npz"), P.random_full_params(6, seed=21))
    out = tmp_path / "tok"
    out.mkdir()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mr_worker.run_existing_dir, args=(r, 2, port, str(pdb_dir), str(mdir), str(out), q))
             for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert got == [(0, "FileExistsError"), (1, "FileExistsError")]
    assert os.listdir(out) == []


def test_global_perplexity_two_ranks():
    """The cross-rank perplexity (one all-reduce) equals the single-process pmean formula."""
    import _mr_worker
    from pst_amd import runner
    rng = np.random.default_rng(5)
    hists = [rng.integers(0, 9, 4096).astype(np.uint32), rng.integers(0, 3, 4096).astype(np.uint32)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mr_worker.run_ppl, args=(r, 2, port, hists, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = runner._perplexity(np.mean([runner._normalised(h) for h in hists], axis=0))
    assert got[0] == got[1]
    assert abs(got[0] - want) <= 1e-9 * want
    assert runner.global_perplexity(hists[0]) == runner._perplexity(runner._normalised(hists[0]))
