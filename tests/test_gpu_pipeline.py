"""pst_tokenize's H2D pipeline (protein chunks copied on a second stream while the previous
chunk computes; the first chunk's copy in protein ranges whose graph kernels start as each range
lands) gives the same bits as the one-shot call: token ids, n_tokens / n_nodes, the
aux outputs and the codebook aux (distances, argmin, histogram) over the whole batch."""
import os

import numpy as np
import pytest

from pst_amd import params as P
from pst_amd import synthetic
from pst_amd._native import pack_samples

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _clear_pipeline_env():
    yield
    for k in ("PST_H2D_CHUNKS", "PST_H2D_GRAPH_RANGES", "PST_H2D_COPY_STREAMS"):
        os.environ.pop(k, None)


def _ctx(chunks, cb=4096, df=1, ranges=None, copy_streams=None):
    """ranges: copy ranges of the first chunk (PST_H2D_GRAPH_RANGES; None = the policy);
    copy_streams: PST_H2D_COPY_STREAMS (2 = odd ranges copied on a second stream). The context
    reads these variables at its FIRST tokenize call, so they stay set until the test ends (or
    the next _ctx call replaces them)."""
    from pst_amd._native import Tokenizer
    os.environ["PST_H2D_CHUNKS"] = str(chunks)
    if copy_streams is None:
        os.environ.pop("PST_H2D_COPY_STREAMS", None)
    else:
        os.environ["PST_H2D_COPY_STREAMS"] = str(copy_streams)
    if ranges is None:
        os.environ.pop("PST_H2D_GRAPH_RANGES", None)
    else:
        os.environ["PST_H2D_GRAPH_RANGES"] = str(ranges)
    return Tokenizer(0, cb, df, P.random_blob(6, 1234))


@pytest.mark.parametrize("cb,df", [(4096, 1), (64000, 4)])
def test_chunked_h2d_is_bitwise_identical(cb, df):
    rng = np.random.default_rng(7)
    lens = [int(x) for x in rng.integers(50, 513, 40)]
    samples = [synthetic.synthetic_protein(n, 900 + i) for i, n in enumerate(lens)]
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    outs = []
    # one copy and one graph launch (the reference point), then the first chunk copied in 4 / 8
    # protein ranges with the graph per range, at 1, 3 and 8 chunks. The batch (~350 tasks) is
    # below the default policy's half-round gate, so the default (None) takes one copy and an
    # explicit PST_H2D_GRAPH_RANGES forces the range branch; the plan each call took is checked.
    # (the first chunk of a forced 3- or 8-chunk plan holds only a few proteins, so it gets at
    # most that many ranges). The last two repeat (1, 4) and (3, 4) with the odd ranges copied on
    # a second stream (PST_H2D_COPY_STREAMS=2): the range events then come from two streams.
    for chunks, ranges, want_ranges, cs in ((1, 1, 0, None), (1, None, 0, None), (1, 4, 4, None), (1, 8, 8, None),
                                            (3, 4, None, None), (8, 8, None, None), (1, 4, 4, 2), (3, 4, None, 2)):
        t = _ctx(chunks, cb, df, ranges, cs)
        tok, nt, nn = t.tokenize_packed(pos, flags, off)
        plan = t.last_plan_detail()
        assert plan["chunks"] == chunks and len(plan["cuts"]) == chunks + 1, (chunks, ranges, plan)
        if want_ranges is None and plan["cuts"][1] == 1:  # one protein: one copy
            assert plan["ranges"] == 0, (chunks, ranges, plan)
        elif want_ranges is None:
            assert 1 <= plan["ranges"] <= min(ranges, plan["cuts"][1]), (chunks, ranges, plan)
        else:
            assert plan["ranges"] == want_ranges, (chunks, ranges, plan)
        tok2, _, _ = t.tokenize_packed(pos, flags, off)  # a second call on the same context
        aux = t.aux(R)
        T = int(nt.sum())
        ca = t.codebook_aux(T, distances=True, soft_proba=cb == 4096)  # 64 000: ~0.7 GB per copy
        outs.append((tok, nt, nn, aux, ca))
        assert np.array_equal(tok, tok2)
        t.close()
    os.environ.pop("PST_H2D_CHUNKS")
    base = outs[0]
    for o in outs[1:]:
        assert np.array_equal(o[0], base[0]) and np.array_equal(o[1], base[1]) and np.array_equal(o[2], base[2])
        for k in ("bounded", "quantize", "pre_proj"):
            assert np.array_equal(o[3][k].view(np.uint32), base[3][k].view(np.uint32)), k
        assert np.array_equal(o[4]["argmin"], base[4]["argmin"])
        assert np.array_equal(o[4]["histogram"], base[4]["histogram"])
        assert np.array_equal(o[4]["distances"].view(np.uint32), base[4]["distances"].view(np.uint32))
        if cb == 4096:
            assert np.array_equal(o[4]["soft_proba"].view(np.uint32), base[4]["soft_proba"].view(np.uint32))


def test_default_pipeline_policy_matches_one_shot():
    """The bench-sized path as it runs by default: 512 proteins x 256 residues = 4 rounds of
    tasks, pipelined as a one-round first chunk (two waves per task) and a three-round rest
    (one wave per task), against one unpipelined call: same token ids and counts."""
    from pst_amd._native import Tokenizer
    samples = synthetic.synthetic_batch(512, 256, seed=4242)
    pos, flags, off = pack_samples(samples)
    os.environ.pop("PST_H2D_CHUNKS", None)
    t = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    tok, nt, nn = t.tokenize_packed(pos, flags, off)
    plan = t.last_plan()
    t.close()
    assert plan == (4, 2)  # default policy: 1 + 3 rounds, first chunk in 4 copy ranges
    t1 = _ctx(1)
    tok1, nt1, nn1 = t1.tokenize_packed(pos, flags, off)
    t1.close()
    os.environ.pop("PST_H2D_CHUNKS")
    assert np.array_equal(tok, tok1) and np.array_equal(nt, nt1) and np.array_equal(nn, nn1)


def test_pipeline_policy_knobs_keep_the_bits(monkeypatch):
    """The remaining schedule knobs the A/B tools set, forced away from their policy values on the
    same inputs, change only the schedule: a first chunk of two rounds growing 2x per chunk with no
    minimum (PST_H2D_FIRST_ROUNDS / PST_H2D_GROWTH / PST_H2D_MIN_ROUNDS: 6 rounds as 2 + 4), and the
    split schedule's edge waves at several blocks per wave (PST_EDGE_WAVES), against unpipelined
    calls: same token ids and counts."""
    from pst_amd._native import Tokenizer
    samples = synthetic.synthetic_batch(768, 256, seed=4343)
    pos, flags, off = pack_samples(samples)
    t1 = _ctx(1)
    tok1, nt1, nn1 = t1.tokenize_packed(pos, flags, off)
    t1.close()
    os.environ.pop("PST_H2D_CHUNKS")
    for k, v in (("PST_H2D_FIRST_ROUNDS", "2"), ("PST_H2D_GROWTH", "2"), ("PST_H2D_MIN_ROUNDS", "1")):
        monkeypatch.setenv(k, v)
    t = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    tok, nt, nn = t.tokenize_packed(pos, flags, off)
    plan = t.last_plan_detail()
    t.close()
    assert plan["chunks"] == 2 and plan["cuts"] == [0, 256, 768], plan
    assert np.array_equal(tok, tok1) and np.array_equal(nt, nt1) and np.array_equal(nn, nn1)
    # split schedule (small batch) with ~4 blocks per edge wave against its default of one
    small = synthetic.synthetic_batch(24, 256, seed=4444)
    spos, sflags, soff = pack_samples(small)
    outs = []
    for ew in (None, "2000"):
        if ew is None:
            monkeypatch.delenv("PST_EDGE_WAVES", raising=False)
        else:
            monkeypatch.setenv("PST_EDGE_WAVES", ew)
        t = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
        outs.append(t.tokenize_packed(spos, sflags, soff))
        assert t.last_plan_detail()["schedules"] == ["split"]
        t.close()
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("chunks", [1, 3])
def test_f32_positions_match_f64(chunks):
    """pst_tokenize_f32 (float32 positions, widened to f64 in k_prep) vs pst_tokenize on the same
    float32-exact values as float64: identical token ids, counts and aux outputs. The batch has
    extra side-chain atoms (centroids over more than the backbone), dropped backbone atoms (gap
    slots) and one protein left with < 50 residues after filtering (the short-protein branch)."""
    rng = np.random.default_rng(11)
    lens = [int(x) for x in rng.integers(52, 400, 12)]
    samples = [synthetic.synthetic_protein(n, 700 + i) for i, n in enumerate(lens)]
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    extra = rng.random(R) < 0.5  # a CB (atom 3) and a CG (atom 5) on half the residues
    for at in (3, 5):
        pos[extra, at] = (pos[extra, 1] + rng.normal(scale=1.5, size=(int(extra.sum()), 3))).astype(np.float32)
        flags[extra, at] = 3
    gaps = rng.random(R) < 0.03
    gaps[int(off[2]):int(off[3])] = False
    flags[gaps, 0] = 0  # missing N: residue dropped
    short = slice(int(off[2]), int(off[2]) + max(0, lens[2] - 49))
    flags[short, 1] = 0  # protein 2 keeps 49 residues
    pos32 = pos.astype(np.float32)
    assert np.array_equal(pos32.astype(np.float64), pos)
    t = _ctx(chunks)
    tok64, nt64, nn64 = t.tokenize_packed(pos, flags, off)
    aux64 = t.aux(R)
    tok32, nt32, nn32 = t.tokenize_packed(pos32, flags, off)
    aux32 = t.aux(R)
    t.close()
    os.environ.pop("PST_H2D_CHUNKS")
    assert nn64[2] == 49
    assert np.array_equal(nt32, nt64) and np.array_equal(nn32, nn64)
    for b in range(len(samples)):
        a = int(off[b])
        assert np.array_equal(tok32[a:a + nt32[b]], tok64[a:a + nt64[b]]), b
    for k in ("bounded", "quantize", "pre_proj"):
        assert np.array_equal(aux32[k].view(np.uint32), aux64[k].view(np.uint32)), k


def test_two_proteins_small_first():
    """A two-protein batch whose first protein is the smaller: the range cut leaves one copy
    range, whose event the graph launch must still wait for (a missing wait raced the copy)."""
    samples = [synthetic.synthetic_protein(60, 41), synthetic.synthetic_protein(480, 42)]
    pos, flags, off = pack_samples(samples)
    outs = []
    # 4 ranges requested on 2 proteins: the cut keeps one range, inside the range branch
    for ranges, plan in ((1, (0, 1)), (4, (1, 1))):
        t = _ctx(1, ranges=ranges)
        for _ in range(3):
            outs.append(t.tokenize_packed(pos, flags, off))
            assert t.last_plan() == plan
        t.close()
    os.environ.pop("PST_H2D_CHUNKS")
    for o in outs[1:]:
        assert np.array_equal(o[1], outs[0][1]) and np.array_equal(o[2], outs[0][2])
        assert list(o[2]) == [60, 480]
        assert np.array_equal(o[0], outs[0][0])


def test_clock_counters_accumulate_and_reset():
    """pst_clock_counters (bench.py's clock fields): off until pst_set_clock_counters enables them;
    then each fused MPNN launch's stamping wave adds
    (shader cycles, 100 MHz ticks) and every wave its lifetime; two calls add about twice one call's
    ticks, reset restarts them, the implied clock is a plausible gfx950 shader clock, the queue
    form's wave-slot occupancy is high (one launch per layer: one chunk), and the tokens are
    unaffected."""
    from pst_amd._native import Tokenizer
    os.environ["PST_H2D_CHUNKS"] = "1"  # one k_mpnn_q launch per layer per call
    samples = synthetic.synthetic_batch(512, 256, seed=1000)  # fused layers (queue form)
    pos, flags, off = pack_samples(samples)
    t = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    tok0, _, _ = t.tokenize_packed(pos, flags, off)
    t.clock_counters(reset=True)
    # off by default: a call stamps nothing until the counters are enabled
    t.tokenize_packed(pos, flags, off)
    z = t.clock_counters()
    assert not z[:, [0, 1, 2, 4, 5]].any() and (z[:, 3] == np.iinfo(np.uint64).max).all()
    t.set_clock_counters(True)
    tok1, _, _ = t.tokenize_packed(pos, flags, off)
    c1 = t.clock_counters().astype(np.float64)
    t.tokenize_packed(pos, flags, off)
    c2 = t.clock_counters(reset=True).astype(np.float64)
    t.close()
    assert np.array_equal(tok0, tok1)
    assert (c1[:, :6] > 0).all(), c1
    span = c1[:, 4] - c1[:, 3]
    occ = c1[:, 2] / (np.minimum(c1[:, 5], 2048) * span)  # queue form: every wave slot, whole launch
    assert ((occ > 0.5) & (occ <= 1.0 + 1e-9)).all(), occ
    c1, c2 = c1[:, :2], c2[:, :2]
    ghz = c1[:, 0] / c1[:, 1] * 0.1
    assert ((ghz > 0.3) & (ghz < 3.0)).all(), ghz
    assert (np.abs(c2[:, 1] / c1[:, 1] - 2.0) < 0.5).all(), (c1, c2)
