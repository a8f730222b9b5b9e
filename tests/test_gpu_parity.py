"""GPU parity: libpst (HIP, through the C ABI) against the CPU oracle, bit for bit.

The canonical numerics make the GPU path and the oracle compute the same
IEEE operation sequence, so every float output is compared BITWISE and token ids exactly.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from pst_amd import params as P
from pst_amd import synthetic
from pst_amd.config import LEVELS

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")

_TOK = {}


def tokenizer(cb=4096, df=1, seed=1234):
    key = (cb, df, seed)
    if key not in _TOK:
        os.environ["PST_DEBUG"] = "1"
        from pst_amd._native import Tokenizer
        _TOK[key] = Tokenizer(0, cb, df, P.random_blob(len(LEVELS[cb]), seed))
    return _TOK[key]


def _samples_from(npz, case):
    from pst_amd.sample import ProteinStructureSample
    pos = npz[case + "/in_positions"].astype(np.float64)
    fl = npz[case + "/in_flags"]
    n = pos.shape[0]
    return ProteinStructureSample(None, n, np.zeros((n, 21)), pos, (fl & 1).astype(bool),
                                  ((fl >> 1) & 1).astype(bool), 0.0, 1)


def _check_batch(samples, cb, df, seed=1234, layers=True):
    tk = tokenizer(cb, df, seed)
    from pst_amd._native import pack_samples
    pos, flags, off = pack_samples(samples)
    tok, nt, nn = tk.tokenize_packed(pos, flags, off)
    R = int(off[-1])
    aux = tk.aux(R)
    feat = tk.debug_fetch(10, R)
    snd = tk.debug_fetch(11, R)
    hl = [tk.debug_fetch(w, R) for w in (1, 2, 3)] if layers else None
    blob = P.random_blob(len(LEVELS[cb]), seed)
    for b, s in enumerate(samples):
        o = O.tokenize(blob, LEVELS[cb], df, s.atom37_positions, s.atom_flags(), want_layers=layers)
        g = o["graph"]
        n = g["n"]
        assert nn[b] == n
        assert nt[b] == n // df
        base = off[b]
        # graph: senders and features bitwise
        gs = snd[base * 50: (base + n) * 50]
        valid = g["senders"] >= 0
        assert np.array_equal(gs[valid] - base, g["senders"][valid])
        gf = feat[base * 50: (base + n) * 50]
        assert np.array_equal(gf.view(np.uint32), g["feat"].view(np.uint32)), "edge features differ"
        if layers:
            for li in range(3):
                got = hl[li][base: base + n]
                want = o["h_layers"][li + 1]
                assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"node features differ after layer {li + 1}: max {np.abs(got - want).max()}"
        T = n // df
        assert np.array_equal(tok[base: base + T], o["tokens"])
        assert np.array_equal(aux["bounded"][base: base + T].view(np.uint32), o["b"].view(np.uint32))
        assert np.array_equal(aux["pre_proj"][base: base + T].view(np.uint32), o["pre_proj"].view(np.uint32))


def test_single_protein_df1():
    _check_batch([synthetic.synthetic_protein(64, 9)], 4096, 1)


def test_ragged_batch_df1():
    F = np.load(os.path.join(GOLD, "forward_golden_f64.npz"))
    samples = [synthetic.synthetic_protein(n, 100 + n) for n in (50, 51, 77, 130, 257)]
    samples.append(_samples_from(F, "syn96_missing_k4096_df1"))
    _check_batch(samples, 4096, 1)


def test_short_protein_branch():
    G = np.load(os.path.join(GOLD, "graph_golden.npz"))
    _check_batch([_samples_from(G, "syn56_missing9_df1"), synthetic.synthetic_protein(50, 3)], 4096, 1)


@pytest.mark.parametrize("cb,df", [(64000, 4), (4096, 2), (432, 1), (1728, 1)])
def test_other_models(cb, df):
    _check_batch([synthetic.synthetic_protein(n, 7 + n) for n in (60, 130, 203)], cb, df, layers=False)


def test_tokens_match_reference_golden():
    """End to end vs the REFERENCE forward (float64 under the shim): identical ids."""
    F = np.load(os.path.join(GOLD, "forward_golden_f64.npz"))
    for case in sorted({k.split("/")[0] for k in F.files}):
        n, T, cb, df, D, seed = (int(v) for v in F[case + "/meta"])
        tk = tokenizer(cb, df, seed)
        toks = tk.tokenize([_samples_from(F, case)])[0]
        assert np.array_equal(toks, F[case + "/tokens"]), case


def test_casp14_batch():
    C = np.load(os.path.join(GOLD, "casp14_atom37.npz"))
    from pst_amd.sample import ProteinStructureSample
    off = C["offsets"]
    samples = []
    for b in range(0, len(off) - 1, 5):  # every 5th protein keeps the CPU oracle fast
        pos = C["positions"][off[b]:off[b + 1]].astype(np.float64)
        fl = C["flags"][off[b]:off[b + 1]]
        n = pos.shape[0]
        samples.append(ProteinStructureSample(None, n, np.zeros((n, 21)), pos, (fl & 1).astype(bool),
                                              ((fl >> 1) & 1).astype(bool), 0.0, 1))
    _check_batch(samples, 4096, 1, layers=False)


def _lattice_protein(side, seed):
    """Identical residues translated onto a side^3 grid (4 A spacing, dyadic atom offsets): the
    centroid distances repeat exactly, so the k-NN selection meets many exact ties at its cut."""
    s = synthetic.synthetic_protein(side ** 3, seed)
    ex = s.atom37_gt_exists[0]
    off = np.round((s.atom37_positions[0] - s.atom37_positions[0, 1]) * 8) / 8
    g = np.stack(np.meshgrid(*[np.arange(side)] * 3, indexing="ij"), -1).reshape(-1, 3) * 4.0
    pos = g[:, None, :] + off[None]
    gt = np.broadcast_to(ex, s.atom37_gt_exists.shape).copy()
    return s._replace(atom37_positions=pos, atom37_gt_exists=gt, atom37_atom_exists=gt.copy())


def test_distance_ties_lattice():
    """Exact distance ties at the neighbour cut resolve to the lower index, as in the oracle."""
    _check_batch([_lattice_protein(4, 2), _lattice_protein(7, 3), _lattice_protein(8, 4)], 4096, 1, layers=False)


def test_size_gates_raise_like_reference():
    tk = tokenizer()
    with pytest.raises(NotImplementedError):
        tk.tokenize([synthetic.synthetic_protein(513, 1)])
    with pytest.raises(NotImplementedError):
        tk.tokenize([synthetic.synthetic_protein(49, 1)])


def test_graph_bitwise_vs_reference_fixtures():
    """Every graph_golden case (reference preprocess_sample run under the shim) in one ragged batch,
    plus a protein whose residues all lack backbone (n = 0): senders and edge features bitwise."""
    G = np.load(os.path.join(GOLD, "graph_golden.npz"))
    cases = sorted(k.split("/")[0] for k in G.files if k.endswith("/n_node"))
    cases = [c for c in cases if int(G[c + "/df"]) == 1]
    samples = [_samples_from(G, c) for c in cases]
    empty = synthetic.synthetic_protein(60, 5)
    gt = empty.atom37_gt_exists.copy()
    gt[:, 4] = False
    ie = len(samples) // 2
    samples.insert(ie, empty._replace(atom37_gt_exists=gt))
    tk = tokenizer(4096, 1)
    from pst_amd._native import pack_samples
    pos, flags, off = pack_samples(samples)
    tok, nt, nn = tk.tokenize_packed(pos, flags, off)
    R = int(off[-1])
    feat = tk.debug_fetch(10, R)
    snd = tk.debug_fetch(11, R)
    gi = 0
    for b, s in enumerate(samples):
        if b == ie:
            assert nn[b] == 0 and nt[b] == 0
            continue
        c = cases[gi]
        gi += 1
        n = int(G[c + "/n_node"])
        assert nn[b] == n, c
        k = 50
        slots = np.arange(n * k)
        r, j = slots // k, slots % k
        deg = min(n, k)
        valid = j < deg
        base = int(off[b])
        got_s = snd[base * k: (base + n) * k] - base
        assert np.array_equal(got_s[valid], G[c + "/senders"][valid]), c
        got_f = feat[base * k: (base + n) * k, :27]
        assert np.array_equal(np.ascontiguousarray(got_f).view(np.uint32), G[c + "/edge_features"].view(np.uint32)), c
    assert gi == len(cases)


@pytest.mark.parametrize("df", [1, 4])
def test_tiny_and_empty_proteins(df):
    """n = 0, 1, 3, 5 usable residues (R = 60 raw each) next to a normal protein."""
    samples = []
    for keep in (0, 1, 3, 5):
        s = synthetic.synthetic_protein(60, 40 + keep)
        gt = s.atom37_gt_exists.copy()
        gt[keep:, 4] = False
        samples.append(s._replace(atom37_gt_exists=gt))
    samples.append(synthetic.synthetic_protein(90, 3))
    cb = 64000 if df == 4 else 4096
    tk = tokenizer(cb, df)
    from pst_amd._native import pack_samples
    pos, flags, off = pack_samples(samples)
    tok, nt, nn = tk.tokenize_packed(pos, flags, off)
    assert nn.tolist() == [0, 1, 3, 5, 90]
    assert nt.tolist() == [n // df for n in (0, 1, 3, 5, 90)]
    blob = P.random_blob(len(LEVELS[cb]), 1234)
    for b, s in enumerate(samples):
        o = O.tokenize(blob, LEVELS[cb], df, s.atom37_positions, s.atom_flags())
        assert np.array_equal(tok[off[b]: off[b] + nt[b]], o["tokens"])


def test_invalid_inputs_rejected():
    import ctypes
    from pst_amd import _native
    tk = tokenizer()
    s = synthetic.synthetic_protein(60, 1)
    pos, flags, off = _native.pack_samples([s, s])
    with pytest.raises(ValueError, match="non-decreasing"):
        tk.tokenize_packed(pos, flags, np.array([0, 60, 50], np.int64))
    with pytest.raises(ValueError, match="prot_offsets\\[0\\]"):
        tk.tokenize_packed(pos, flags, np.array([1, 61, 120], np.int64))
    with pytest.raises(ValueError):
        tk.tokenize_packed(pos, flags, np.array([0], np.int64))  # empty batch
    L = _native.lib()
    nt = np.zeros(2, np.int32)
    rc = L.pst_tokenize(tk._h, None, _native._ptr(flags), _native._ptr(off), 2, None, _native._ptr(nt), None)
    assert rc == _native.PST_E_INVALID
    # the context still works after rejected calls
    assert np.array_equal(tk.tokenize([s])[0], O.tokenize(P.random_blob(6, 1234), LEVELS[4096], 1, s.atom37_positions, s.atom_flags())["tokens"])


@pytest.mark.parametrize("split,half,queue", [("0", "0", "0"), ("0", "1", "0"), ("1000000", "0", "0"),
                                              ("0", "0", "1")])
def test_fused_and_split_layers_identical(split, half, queue, monkeypatch):
    """The MPNN schedules (fused: one wave per 32 receivers; fused with two waves per task, 16
    receivers each; split: edge blocks spread over the GPU, messages through HBM; fused as the
    persistent half-task queue, k_mpnn_q) give the same bits. Small batches default to split, so
    this forces each mode in a fresh context and compares with the oracle-checked default."""
    from pst_amd._native import Tokenizer, pack_samples
    samples = [synthetic.synthetic_protein(n, 300 + n) for n in (50, 99, 256, 512, 131)]
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    ref = tokenizer(4096, 1, 1234)  # default policy (fixed at a context's first call)
    tok2, _, _ = ref.tokenize_packed(pos, flags, off)
    hl2 = [ref.debug_fetch(w, R) for w in (1, 2, 3)]
    monkeypatch.setenv("PST_SPLIT_TASKS", split)
    monkeypatch.setenv("PST_HALF_TASKS", half)
    monkeypatch.setenv("PST_MPNN_QUEUE", queue)
    monkeypatch.setenv("PST_DEBUG", "1")
    tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    tok, nt, nn = tk.tokenize_packed(pos, flags, off)
    if queue == "1":
        assert tk.last_plan_detail()["schedules"] == ["fused_queue"]
    hl = [tk.debug_fetch(w, R) for w in (1, 2, 3)]
    for a, b in zip(hl, hl2):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(tok[:R], tok2[:R])
    blob = P.random_blob(6, 1234)
    s = samples[2]
    o = O.tokenize(blob, LEVELS[4096], 1, s.atom37_positions, s.atom_flags())
    assert np.array_equal(tok[off[2]: off[2] + nt[2]], o["tokens"])


@pytest.mark.parametrize("cb", [4096, 64000])
def test_down_coop_and_one_wave_identical(cb, monkeypatch):
    """k_down_coop (four waves per 32-token tile, small batches), k_down_pair (two waves per
    tile, one track each, one-round batches) and k_down<1> (one wave per tile) give the same bits:
    tokens, bounded/quantized codes and pre-projection embeddings. Odd tile count (the pair
    kernel's last workgroup holds one live tile) and ragged proteins."""
    from pst_amd._native import Tokenizer, pack_samples
    samples = [synthetic.synthetic_protein(n, 700 + n) for n in (51, 64, 200, 512, 97)]
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    blob = P.random_blob(len(LEVELS[cb]), 77)
    outs = []
    for coop, pair, form in (("0", "0", "one_wave"), ("1000000", "0", "coop"), ("0", "1", "pair")):
        monkeypatch.setenv("PST_DOWN_COOP", coop)
        monkeypatch.setenv("PST_DOWN_PAIR", pair)
        monkeypatch.setenv("PST_H2D_CHUNKS", "1")
        tk = Tokenizer(0, cb, 1, blob)
        tok, nt, _ = tk.tokenize_packed(pos, flags, off)
        assert tk.last_plan_detail()["downsampler"] == form
        outs.append((tok[:R].copy(), tk.aux(R)))
        tk.close()
    t0, a0 = outs[0]
    for t1, a1 in outs[1:]:
        assert np.array_equal(t0, t1)
        for k in ("bounded", "quantize", "pre_proj"):
            assert np.array_equal(a0[k].view(np.uint32), a1[k].view(np.uint32)), k
    s = samples[3]
    o = O.tokenize(blob, LEVELS[cb], 1, s.atom37_positions, s.atom_flags())
    assert np.array_equal(outs[2][0][off[3]: off[3] + nt[3]], o["tokens"])


def test_node_coop_and_one_wave_identical(monkeypatch):
    """Split schedule: k_mpnn_node_coop (four waves per 32 receivers) and k_mpnn_node (one wave)
    give the same node features after every layer and the same tokens."""
    from pst_amd._native import Tokenizer, pack_samples
    samples = [synthetic.synthetic_protein(n, 900 + n) for n in (50, 77, 256, 512, 130)]
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    blob = P.random_blob(6, 1234)
    monkeypatch.setenv("PST_SPLIT_TASKS", "1000000")
    monkeypatch.setenv("PST_DEBUG", "1")
    outs = []
    for coop in ("0", "1000000"):
        monkeypatch.setenv("PST_NODE_COOP", coop)
        tk = Tokenizer(0, 4096, 1, blob)
        tok, nt, _ = tk.tokenize_packed(pos, flags, off)
        outs.append((tok[:R].copy(), [tk.debug_fetch(w, R) for w in (1, 2, 3)]))
    (t0, h0), (t1, h1) = outs
    for a, b in zip(h0, h1):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(t0, t1)
    s = samples[2]
    o = O.tokenize(blob, LEVELS[4096], 1, s.atom37_positions, s.atom_flags())
    assert np.array_equal(t1[off[2]: off[2] + nt[2]], o["tokens"])


def test_build_graph_matches_reference_padded_graphs():
    """pst_build_graph + the host padding == the reference's preprocess_sample(...).graph for
    every graph_golden case, in one ragged batch (edge features bitwise as float32)."""
    from test_graph_host import CASES, PG, check_graph
    from pst_amd import graph as Gr
    G = np.load(os.path.join(GOLD, "graph_golden.npz"))
    by_df = {}
    for c in CASES:
        by_df.setdefault(int(G[c + "/df"]), []).append(c)
    tk = tokenizer(4096, 1)
    for df, cases in by_df.items():
        graphs = Gr.build_protein_graphs(tk, [_samples_from(G, c) for c in cases], df)
        for c, g in zip(cases, graphs):
            check_graph(g, c)
    # the tokenize path still works on the same context afterwards
    s = synthetic.synthetic_protein(64, 9)
    assert np.array_equal(tk.tokenize([s])[0], O.tokenize(P.random_blob(6, 1234), LEVELS[4096], 1, s.atom37_positions, s.atom_flags())["tokens"])


def test_make_graph_from_pdb_reads_as_reference_graph(tmp_path):
    """runner.make_graph_from_pdb on CASP14 T1024: the returned view's ProteinGraph fields equal
    the reference's graph of the same file."""
    import tarfile
    from test_graph_host import check_graph
    from pst_amd import runner
    with tarfile.open(os.path.join(GOLD, "casp14_pdbs.tar.gz")) as tf:
        m = [x for x in tf.getmembers() if x.name.endswith("T1024.pdb")][0]
        tf.extract(m, tmp_path)
    v = runner.make_graph_from_pdb(str(tmp_path / m.name), num_neighbor=50, downsampling_ratio=1,
                                   residue_loc_is_alphac=True, padding_num_residue=512)
    check_graph(v.graph, "casp_T1024_df1")
    assert np.array_equal(v.senders, v.graph.senders) and v.nb_residues == 391


def test_mpnn_queue_identical_at_full_rounds(monkeypatch):
    """k_mpnn_q at several rounds of tasks (3 072 tasks, ragged proteins so tasks straddle
    proteins): the halves of a task are handed between waves that may sit on different XCDs
    (agent release / acquire); node features after every layer, tokens and bounded latents must
    equal the one-wave fused form bit for bit, on three calls of the same context (L1/L2 warm,
    the counters re-zeroed per call)."""
    from pst_amd._native import Tokenizer, pack_samples
    rng = np.random.default_rng(5)
    lens = [int(x) for x in rng.integers(60, 513, 340)]
    samples = [synthetic.synthetic_protein(n, 4000 + i) for i, n in enumerate(lens)]
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    outs = []
    monkeypatch.setenv("PST_DEBUG", "1")
    monkeypatch.setenv("PST_H2D_CHUNKS", "1")
    # queue on every layer (the default since round 6) with the default unit order (groups of one
    # XCD's wave slots), with adjacent halves (group 0), layers 1-2 only (the round-4 default, layer 0
    # one wave per task) with a group size that leaves a partial group in every XCD's range
    # (3 072 / 8 = 384 tasks = 10 x 37 + 14), and the 4-wave queue workgroups
    for queue, layers, group, qw in (("0", "-", "-", "-"), ("1", "7", "-", "-"), ("1", "7", "0", "-"),
                                     ("1", "6", "37", "-"), ("1", "-", "-", "4")):
        monkeypatch.setenv("PST_MPNN_QUEUE", queue)
        for k, v in (("PST_MPNN_QUEUE_LAYERS", layers), ("PST_MPNN_QGROUP", group), ("PST_MPNN_QWAVES", qw)):
            if v == "-":
                monkeypatch.delenv(k, raising=False)
            else:
                monkeypatch.setenv(k, v)
        tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
        for rep in range(3 if (layers == "7" and group == "-") else 1 if queue == "0" else 2):
            tok, nt, nn = tk.tokenize_packed(pos.astype(np.float32), flags, off)
            assert tk.last_plan_detail()["schedules"] == (["fused_queue"] if queue == "1" else ["fused"])
            hl = [tk.debug_fetch(w, R) for w in (1, 2, 3)]
            outs.append((tok[:R].copy(), [h.view(np.uint32).copy() for h in hl], tk.aux(R)["bounded"].view(np.uint32)))
        tk.close()
    base = outs[0]
    for o in outs[1:]:
        assert np.array_equal(o[0], base[0])
        for a, b in zip(o[1], base[1]):
            assert np.array_equal(a, b)
        assert np.array_equal(o[2], base[2])


@pytest.mark.parametrize("lens", [(50,), (50, 51), (130, 77, 301, 52, 64)])
def test_mpnn_queue_forced_on_small_batches(lens, monkeypatch):
    """The persistent queue forced onto batches far below one round (4 to 20 tasks: most XCD
    ranges empty, a wave finds its own queue empty and steals from the others; the unit group larger
    than a range) on every layer, with the default unit order, with adjacent halves and with 4-wave
    workgroups: node features after every layer and tokens equal the default schedule's bit for
    bit."""
    from pst_amd._native import Tokenizer, pack_samples
    samples = [synthetic.synthetic_protein(n, 5100 + i) for i, n in enumerate(lens)]
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    monkeypatch.setenv("PST_DEBUG", "1")
    ref = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    tok0, _, _ = ref.tokenize_packed(pos, flags, off)
    h0 = [ref.debug_fetch(w, R).view(np.uint32).copy() for w in (1, 2, 3)]
    ref.close()
    for env in ({"PST_MPNN_QUEUE_LAYERS": "7"}, {"PST_MPNN_QUEUE_LAYERS": "7", "PST_MPNN_QGROUP": "0"},
                {"PST_MPNN_QUEUE_LAYERS": "7", "PST_MPNN_QWAVES": "4"}):
        monkeypatch.setenv("PST_SPLIT_TASKS", "0")
        monkeypatch.setenv("PST_HALF_TASKS", "0")
        monkeypatch.setenv("PST_MPNN_QUEUE", "1")
        for k in ("PST_MPNN_QUEUE_LAYERS", "PST_MPNN_QGROUP", "PST_MPNN_QWAVES"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
        tok, _, _ = tk.tokenize_packed(pos, flags, off)
        assert tk.last_plan_detail()["schedules"] == ["fused_queue"]
        for w, b in zip((1, 2, 3), h0):
            assert np.array_equal(tk.debug_fetch(w, R).view(np.uint32), b), (env, w)
        assert np.array_equal(tok[:R], tok0[:R]), env
        tk.close()

