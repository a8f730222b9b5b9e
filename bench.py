"""Benchmark: residues tokenized/s (codebook 4096, df 1) on MI355X — BASELINE.json's metric.

Workload (SURVEY config 3): 1 024 synthetic proteins × 256 residues = 262 144 residues, K = 4096,
df = 1, batch-sharded over the N GPUs of the job (LPT on residues: 128 proteins per GPU at N = 8;
"scaling": "strong", total work fixed). `--weak` instead gives every GPU its own 1 024 proteins.

One step = one tokenization of the rank's whole batch with its inputs already resident in HBM
(the task's `value` contract): atom37 positions (float64) + flags in device memory → graph build
→ 3 MPNN layers → downsampler → FSQ → token ids in device memory (`pst_tokenize_device`,
synchronised per step). W warm-up steps, then K timed steps bracketed by barrier + synchronize;
each step is also timed on its own, the per-step time is the max over ranks, `ms_per_step` is the
median of the K and `value` = all residues of the job / that median.

Reported beside it, never as `value`: BASELINE.md §4's PCIe-inclusive region (`host_to_host`):
atom37 in pinned host memory → H2D → … → D2H token ids (`pst_tokenize_f32`, the PDB path's float32
coordinates; `--f64-input` times `pst_tokenize` on float64 arrays, and the other format is
reported beside it; libpst pipelines the H2D of protein chunks with the compute), K steps, median,
max over ranks. Its tokens must equal the device-resident step's (checked).

Launch: `python bench.py` (1 GPU); `python bench.py --gpus N` spawns N worker processes itself
(the parent never touches the GPU); under `torch.distributed.run` each rank is one GPU (RCCL for
the barrier and the max-over-ranks reductions; no collective on the data path).

Also reported on rank 0: the dominant kernel's
roofline from HIP events on the library's stream (executed MFMA FLOPs / launch time / f32 MFMA
peak), per-kernel fractions, exact match vs the reference's own forward on the fixture proteins
of the workload (tests/golden/forward_ref_wide.npz) and vs the C oracle, the CPU baselines
(the reference's computation as it is done — padded, dense — in PyTorch-CPU, and the ragged C
port) and the CASP14 CLI end-to-end figure.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "tests", "golden"), ROOT, os.path.join(ROOT, "protein-structure-tokenizer_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

N_PROT, N_RES, CODEBOOK, DF = 1024, 256, 4096, 1
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense f32 MFMA (and packed-f32 VALU) peak
SPEC_GHZ = 2.4             # the shader clock the peak is quoted at
H, K = 128, 50
MFMA_FLOP = 32 * 32 * 2 * 2  # one v_mfma_f32_32x32x2_f32
# MFMA instructions per 32-receiver task (equal to the PMC SQ_INSTS_MFMA per launch
# / (R/32), profiles/r02_pmc_mfma.txt): per 32-edge block k_mpnn<0> 372 (edge embed 14·4 +
# message first layer 14·4 over the 27 features in 14 k-steps + W1 65·4; 380 with 15 k-steps
# before round 5), k_mpnn<1,2> 1292 (edge MLP 64·4 + 65·4 + 65·4, message MLP 64·4 + 65·4); node
# part: message W2 after the segment sum 256, FFN 2068, projections 1032 (layers 0, 1 only).
MFMA_PER_TASK = {"mpnn0": 50 * 372 + 256 + 2068 + 1032, "mpnn1": 50 * 1292 + 256 + 2068 + 1032,
                 "mpnn2": 50 * 1292 + 256 + 2068}
# SURVEY §8d algorithmic FLOPs (padding and dead code removed) of k_mpnn<1>'s work: edge MLP of
# layer 1 + message MLP of layer 2 over 50 edges + the layer-2 node FFN
MLP_FLOP = 2 * (3 * H * H + H * H + H * H)
MPNN1_ALG_FLOP_PER_RES = K * 2 * MLP_FLOP + 2 * (H * 4 * H + 4 * H * H)   # 16 646 144
PATH_ALG_FLOP_PER_RES = {1: 44_715_008, 4: 44_395_904}  # SURVEY §8d, whole path per residue


T0 = time.perf_counter()


def log(msg: str) -> None:
    """Progress on stderr (the JSON line stays alone on stdout)."""
    print(f"[bench {time.perf_counter() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def host_cores() -> int:
    """CPU threads this process may really use: the affinity set, capped by the cgroup CPU quota
    (a GPU box shows the whole machine's CPUs but grants a share) and by OMP_NUM_THREADS."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(-(-int(q) // int(per)))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--proteins", type=int, default=N_PROT, help="proteins of the whole job (per GPU with --weak)")
    ap.add_argument("--residues", type=int, default=N_RES)
    ap.add_argument("--weak", action="store_true", help="every GPU runs --proteins proteins of its own")
    ap.add_argument("--codebook", type=int, default=CODEBOOK, help="secondary configs (default: the metric's 4096)")
    ap.add_argument("--df", type=int, default=DF)
    ap.add_argument("--f64-input", action="store_true",
                    help="time pst_tokenize on float64 positions instead of pst_tokenize_f32 on float32 ones")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the CASP14 end-to-end field")
    ap.add_argument("--cpu-sample", type=int, default=64,
                    help="proteins in the reference-as-computed CPU sample (spread over the workload)")
    ap.add_argument("--port-sample", type=int, default=128, help="proteins in the C-port CPU sample")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_k_mpnn1.json"),
                    help="PMC-measured HBM bytes per residue of k_mpnn<1> (tools/pmc_traffic.sh)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, the driver's runs) or gloo (rehearsing several ranks on one GPU)")
    ap.add_argument("--plan", action="store_true", help="launch + rendezvous (gloo) + sharding only, no GPU")
    return ap.parse_args()


def spawn_workers(n: int) -> int:
    """`bench.py --gpus N` without a launcher: N child processes, one per GPU (RANK/LOCAL_RANK/
    WORLD_SIZE set here); rank 0 prints the JSON line. This process never initialises the GPU."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # wait for every child; once one fails, the others may be blocked in a collective with it,
    # so they get a grace period and are then terminated (never left holding a GPU)
    import time
    failed_at = None
    while any(p.poll() is None for p in procs):
        if failed_at is None and any(p.returncode not in (None, 0) for p in procs):
            failed_at = time.monotonic()
        if failed_at is not None and time.monotonic() - failed_at > 30:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=15)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    codes = [p.wait() for p in procs]
    return next((c for c in codes if c != 0), 0)


def init_group(backend: str, **kw) -> None:
    """dist.init_process_group with the gloo transport's connection banner (printed on the
    process's stdout) sent to stderr: stdout carries only the JSON line."""
    import torch.distributed as dist
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group(backend, **kw)
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def shard_ids(args, rank, world):
    """Protein ids of this rank (protein p is synthetic_protein(residues, seed 1000 + p))."""
    from pst_amd import runner
    if args.weak:
        return [rank * args.proteins + p for p in range(args.proteins)]
    return runner.lpt_partition([args.residues] * args.proteins, world)[rank]


def workload(args, rank, world):
    from pst_amd import synthetic
    ids = shard_ids(args, rank, world)
    return ids, [synthetic.synthetic_protein(args.residues, 1000 + p) for p in ids]


def plan_only(args, rank, world):
    """--plan: the launch, rendezvous and sharding of a run without touching a GPU (gloo).
    Rank 0 prints what the run would process."""
    import torch
    import torch.distributed as dist
    if world > 1:
        init_group("gloo")
    ids = shard_ids(args, rank, world)
    t = torch.tensor([len(ids), len(ids) * args.residues], dtype=torch.int64)
    allids = [None] * world
    if world > 1:
        dist.all_reduce(t)
        dist.all_gather_object(allids, ids)
    else:
        allids = [ids]
    if rank == 0:
        print(json.dumps({"n_gpus": world, "world_size_seen": dist.get_world_size() if world > 1 else 1,
                          "proteins_job": int(t[0]), "residues_job": int(t[1]),
                          "proteins_per_rank": [len(x) for x in allids],
                          "disjoint": len(set(sum(allids, []))) == sum(len(x) for x in allids),
                          "scaling": "weak" if args.weak else "strong"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def reference_exact_match(args, ids, tok, off, plan=None, bounded=None):
    """Token ids of this rank's proteins vs the reference's own forward (Vq3D.encode_and_quantize
    under the shim, float64 with JAX's float32 PE argument, i.e. the reference's PE values):
    tests/golden/forward_ref_bench.npz holds EVERY protein of the headline workload (bench256:
    1 024 proteins, 262 144 tokens) and of config 5's (bench512: 512 proteins, 65 536 tokens), with
    per-token margins, the bounded latents of the close tokens and every latent of a 32-protein
    subset of each workload (refwide.BenchSample). Every mismatch is listed with
    its protein, token, latent dim, the reference's margin and our deviation; with `bounded` (our
    FSQ-bounded latents, pst_aux) the report carries our deviation on every close token."""
    try:
        import refwide
    except Exception:
        return None
    name = {(4096, 1, 256): "bench256", (64000, 4, 512): "bench512"}.get((args.codebook, args.df, args.residues))
    if name is None:
        return None
    try:
        S = refwide.load_bench_sample(name)
    except Exception:
        return None
    pos_of = {p: i for i, p in enumerate(ids)}
    prots = [p for p in ids if p in S.index]
    if not prots:
        return None
    sl = [slice(int(off[pos_of[p]]), int(off[pos_of[p]]) + S.n_tokens(p)) for p in prots]
    r = S.compare(prots, [tok[x] for x in sl], [bounded[x] for x in sl] if bounded is not None else None)
    cuts = plan["cuts"] if plan else None
    by_chunk = {}
    for p, x in zip(prots, sl):
        k = str(int(np.searchsorted(cuts, pos_of[p], side="right") - 1)) if cuts else "0"
        b = by_chunk.setdefault(k, {"proteins": 0, "tokens": 0, "identical": 0})
        b["proteins"] += 1
        b["tokens"] += x.stop - x.start
        b["identical"] += int(np.sum(tok[x] == S.ref_tokens(p)))
    return {"proteins_compared": r["proteins"], "proteins_in_workload": len(ids), "tokens_compared": r["tokens"],
            "identical": r["identical"], "rate": r["rate"], "by_pipeline_chunk": by_chunk,
            "min_margin": r["min_margin"], "close_tokens": r["close_tokens"], "close_below": r["close_below"],
            "max_deviation_close": r["max_deviation_close"],
            "max_deviation_over_margin_close": r["max_deviation_over_margin_close"],
            "full_latent_proteins": r["full_latent_proteins"], "max_deviation_full": r["max_deviation_full"],
            "mismatches": r["mismatches"], "mismatches_explained_by_rounding": r["mismatches_explained_by_rounding"],
            "unlisted_mismatches": len(r["unlisted"]), "known_cases_not_flipped": r["missing_known"],
            "margin_histogram_all": r["margin_histogram_all"],
            "margin_histogram_mismatches": r["margin_histogram_mismatches"],
            "against": "reference Vq3D.encode_and_quantize run in float64 under the shim with JAX's float32 "
                       f"PE argument (tests/golden/forward_ref_bench.npz '{name}': {len(S)} proteins of the workload, "
                       "make_forward_bench.py + compact_bench.py)"}


def clock_stats(per_step, steps=None):
    """Shader clock from libpst's clock counters (pst_clock_counters): the stamping wave of each
    fused MPNN launch contributes (s_memtime cycles, s_memrealtime 100 MHz ticks); clock = cycles /
    ticks x 0.1 GHz over the three layers (~90 % of a step's device time). `per_step`: one record
    per read — per step (min / max over them), or one read summed over `steps` steps (the timed
    loop reads once, after it). Mean (cycle-weighted), per-layer means."""
    if not per_step:
        return None
    c = np.array(per_step, np.float64)[:, :, :2]  # [steps, 3, (cycles, ticks)]
    if c[..., 1].sum() <= 0:
        return None
    step = c[:, :, 0].sum(1) / np.maximum(c[:, :, 1].sum(1), 1) * 0.1
    layer = c[:, :, 0].sum(0) / np.maximum(c[:, :, 1].sum(0), 1) * 0.1
    out = {"mean_ghz": round(float(c[..., 0].sum() / c[..., 1].sum() * 0.1), 4),
           "per_layer_ghz": [round(float(x), 4) for x in layer], "steps": steps or len(per_step),
           "stamped_ms": round(float(c[..., 1].sum() / 1e5), 1)}
    if len(per_step) > 1:
        out.update(min_ghz=round(float(step.min()), 4), max_ghz=round(float(step.max()), 4))
    else:
        out["read"] = "once, summed over the timed steps"
    return out


def wave_slot_occupancy(per_step, slots):
    """Wave-slot occupancy of each MPNN layer launch (one launch per layer per step): the sum of
    its waves' lifetimes over slots x (last end - first start), from the same clock counters
    (clk[2] lifetimes, clk[3] min start, clk[4] max end, 100 MHz ticks). 1 - occupancy is the
    launch's idle slot time: ramp, tail and any slot a wave leaves empty."""
    if not per_step:
        return None
    c = np.array(per_step, np.float64)  # [steps, 3, 8]
    span = c[:, :, 4] - c[:, :, 3]
    if (span <= 0).any():
        return None
    occ = (c[:, :, 2] / (slots * span)).mean(0)
    return {"per_layer": [round(float(x), 4) for x in occ], "slots": int(slots),
            "waves_per_launch": [int(x) for x in c[0, :, 5]]}


def casp14_end_to_end(tk):
    """SURVEY config 2 as the CLI runs it (InferenceRunner.tokenize's libpst path): read the 31
    CASP14 PDB files, parse them on the GPU and tokenize (pst_tokenize_pdb_files: the texts go to
    HBM, the atom37 rows never return to the host), write <stem>_tokens.npy. Reported beside
    `value`, with the same step through the native host parser for comparison."""
    import tarfile
    import tempfile
    from pst_amd._native import parse_pdb_files, parse_pdb_files_handle
    from pst_amd.runner import save_npy_files
    arc = os.path.join(ROOT, "tests", "golden", "casp14_pdbs.tar.gz")
    if not os.path.exists(arc):
        return None, None
    threads = min(16, host_cores())
    # inputs and token files on tmpfs where there is one: the figure is the software path (read,
    # parse, H2D + tokenize, .npy encode + write syscalls), not the speed of the box's disk
    shm = "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else None
    with tempfile.TemporaryDirectory(dir=shm) as d:
        with tarfile.open(arc) as tf:
            tf.extractall(d, members=[m for m in tf.getmembers() if m.isfile() and m.name.endswith(".pdb")])
        files = sorted(os.path.join(d, "casp14_pdbs", f) for f in os.listdir(os.path.join(d, "casp14_pdbs")))
        names = [os.path.basename(f)[:-4] + "_tokens" for f in files]
        runs, host_runs = [], []
        for rep in range(7):  # first pass warms the page cache and the context's buffers
            out = os.path.join(d, f"out{rep}")
            os.makedirs(out)
            t0 = time.perf_counter()
            tok, nt, _, off = tk.tokenize_pdb_files(files, n_threads=threads)
            t1 = time.perf_counter()
            save_npy_files([os.path.join(out, nm) for nm in names],
                           [tok[int(off[i]):int(off[i]) + nt[i]].reshape(1, -1) for i in range(len(files))])
            t2 = time.perf_counter()
            if rep:
                runs.append((t2 - t0, t1 - t0, t2 - t1))
            gpu_files = len(files) - tk.pdb_files_host_parsed()
            # the same step with the native host parser (pst_pdb_parse_files + pst_tokenize_pdb_batch)
            hout = os.path.join(d, f"hout{rep}")
            os.makedirs(hout)
            t0 = time.perf_counter()
            H = parse_pdb_files_handle(files, n_threads=threads)
            t1 = time.perf_counter()
            htok, hnt, _ = tk.tokenize_pdb_batch(H)
            hoff = H.offsets()
            H.close()
            t2 = time.perf_counter()
            save_npy_files([os.path.join(hout, nm) for nm in names],
                           [htok[int(hoff[i]):int(hoff[i]) + hnt[i]].reshape(1, -1) for i in range(len(files))])
            t3 = time.perf_counter()
            if rep:
                host_runs.append((t3 - t0, t1 - t0, t2 - t1, t3 - t2))
        assert np.array_equal(off, hoff) and np.array_equal(nt, hnt)
        same = all(np.array_equal(tok[int(off[i]):int(off[i]) + nt[i]], htok[int(off[i]):int(off[i]) + nt[i]])
                   for i in range(len(files)))
        B = parse_pdb_files(files, n_threads=threads, float32=True)  # arrays for the CPU baseline
        R = int(B.offsets[-1])
        casp = (B.positions.astype(np.float64), np.array(B.flags), np.array(B.offsets), (htok.copy(), np.array(hnt)))
        tot, rpt, write = runs[int(np.argsort([r[0] for r in runs])[len(runs) // 2])]  # median run
        htot, hparse, htokz, hwrite = host_runs[int(np.argsort([r[0] for r in host_runs])[len(host_runs) // 2])]
        res = {"workload": "CASP14 31 structures (SURVEY config 2), codebook 4096, df 1", "residues": R,
               "read_parse_tokenize_ms": round(rpt * 1e3, 2), "write_ms": round(write * 1e3, 2),
               "residues_per_s": round(R / tot, 1), "files_parsed_on_gpu": gpu_files,
               "path": "pst_tokenize_pdb_files (files read on the host pool into page-locked memory, text to HBM, "
                       "parse on the GPU, tokenize) + native token-file writer",
               "host_parser_path": {"parse_ms": round(hparse * 1e3, 2), "tokenize_ms": round(htokz * 1e3, 2),
                                    "write_ms": round(hwrite * 1e3, 2), "residues_per_s": round(R / htot, 1),
                                    "tokens_identical": bool(same)},
               "threads": threads, "runs": f"median of {len(runs)} after one warm-up",
               "files_on": shm or tempfile.gettempdir()}
    return res, casp


def _ref_as_computed_rate(model, pf, df, threads, cores, what):
    """Time the reference-as-computed PyTorch-CPU forward one protein per call (the reference CLI's
    batch_size_per_device default), graphs padded as the reference pads them."""
    import torch
    from oracle.reference_as_computed import padded_graphs
    torch.set_num_threads(threads)
    model.forward(padded_graphs(pf[:1], model.df))  # warm-up
    res_n = int(sum(p.shape[0] for p, _ in pf))
    toks = []
    t0 = time.perf_counter()
    for i in range(len(pf)):
        toks.append(model.forward(padded_graphs(pf[i:i + 1], df))["tokens"][0])
    dt = time.perf_counter() - t0
    return {"value": round(res_n / dt, 1), "unit": "residues/s", "cores": threads, "kind": "port",
            "sample": f"{what} ({len(pf)} proteins, {res_n} residues), {dt:.1f} s: the reference's computation as it "
                      "runs it (graph padded to 512 nodes / 25 600 edges, per-edge PE, dense masked cross-attention, "
                      "FSQ distances/soft_proba over all K), PyTorch-CPU float32 (oracle/reference_as_computed.py) + "
                      f"the C graph, one protein per call; torch.set_num_threads({threads}) of {cores} cores available"}, toks


def _reference_sample(args):
    """refwide.BenchSample of this workload (None when there is none)."""
    name = {(4096, 1, 256): "bench256", (64000, 4, 512): "bench512"}.get((args.codebook, args.df, args.residues))
    try:
        import refwide
        return refwide.load_bench_sample(name) if name else None
    except Exception:
        return None


def cpu_baselines(args, samples, blob, levels, pos, flags, off, gpu_tok, plan=None, casp=None, ref_ids=None):
    """CPU baselines (reported, not targeted): the reference-as-computed PyTorch-CPU
    forward on a `--cpu-sample`-protein subset of the workload (every 16th protein by default, so
    both pipeline chunks) and on SURVEY config 2 (the 31 CASP14 structures, `casp` = (positions,
    flags, offsets, GPU tokens) from casp14_end_to_end), each at all allowed cores and at 8 threads;
    the ragged C port; and the GPU-vs-C-oracle exact match on the port's sample."""
    import torch
    from oracle import oracle as O
    from oracle.reference_as_computed import ReferenceAsComputed
    from pst_amd import params as P
    cores = host_cores()
    model = ReferenceAsComputed(P.random_params(len(levels), 1234), levels, args.df)
    nb = len(samples)
    n = min(args.cpu_sample, nb)
    csel = np.arange(0, nb, max(1, nb // max(1, n)))[:n]
    pf = [(samples[i].atom37_positions, samples[i].atom_flags()) for i in csel]
    out = {}
    for threads in sorted({cores, 8}, reverse=True):
        log(f"reference-as-computed CPU baseline (config 3 subset), {threads} threads, {len(pf)} proteins")
        out[threads], toks = _ref_as_computed_rate(model, pf, args.df, threads, cores,
                                                   f"every {max(1, nb // max(1, n))}th protein of the workload")
        # protein i's T = n_i / df tokens sit at gpu_tok[off[i] .. off[i] + T) (raw-offset layout)
        ms = [min(len(t), int(off[i + 1] - off[i]) // args.df) for t, i in zip(toks, csel)]
        ident = sum(int(np.sum(t[:m] == gpu_tok[off[i]:off[i] + m])) for t, i, m in zip(toks, csel, ms))
        out[threads]["tokens_identical_to_gpu"] = f"{ident} / {sum(ms)}"
        # against the reference itself: PyTorch-CPU float32 reduces in a thread-count-dependent
        # order, so a token whose reference margin is below its deviation may flip in one setting
        # and not another; every difference is listed with its reference margin
        ref = _reference_sample(args)
        if ref is not None:
            import refwide
            ids_s = [ref_ids[i] for i in csel] if ref_ids is not None else list(csel)
            keep = [k for k, p in enumerate(ids_s) if p in ref.index]
            rr = ref.compare([ids_s[k] for k in keep], [toks[k][:ref.n_tokens(ids_s[k])] for k in keep],
                             known=refwide.KNOWN_CPU_BASELINE_CASES)
            out[threads]["tokens_identical_to_reference"] = f"{rr['identical']} / {rr['tokens']}"
            out[threads]["mismatches_vs_reference"] = [
                {k: m[k] for k in ("protein", "token", "ref_margin", "dim") if k in m} for m in rr["mismatches"]]
            out[threads]["unexplained_vs_reference"] = len(rr["unexplained"])
            # every flip must be a listed known case (refwide.KNOWN_CPU_BASELINE_CASES), and every
            # listed case of the sample must still flip
            out[threads]["unlisted_vs_reference"] = len(rr["unlisted"])
            out[threads]["known_cases_not_flipped"] = rr["missing_known"]
    cfg2 = {}
    if casp is not None and args.codebook == 4096 and args.df == 1:
        cpos, cflags, coff, ctok = casp
        cpf = [(cpos[coff[i]:coff[i + 1]], cflags[coff[i]:coff[i + 1]]) for i in range(len(coff) - 1)]
        for threads in sorted({cores, 8}, reverse=True):
            log(f"reference-as-computed CPU baseline (config 2, CASP14), {threads} threads")
            cfg2[threads], toks = _ref_as_computed_rate(model, cpf, args.df, threads, cores,
                                                        "SURVEY config 2: the 31 CASP14 structures")
            if threads == max(cores, 8):
                eq = tot = 0
                for i, t in enumerate(toks):
                    m = int(ctok[1][i])
                    eq += int(np.sum(t[:m] == ctok[0][coff[i]:coff[i] + m]))
                    tot += m
                cfg2[threads]["tokens_identical_to_gpu"] = f"{eq} / {tot}"
    torch.set_num_threads(cores)
    # the C-port sample is spread over the whole workload (every stride-th protein), so it checks
    # every pipeline chunk the timed step runs, not only the first
    stride = max(1, -(-nb // max(1, args.port_sample)))
    sel = np.arange(0, nb, stride)
    lens = off[sel + 1] - off[sel]
    soff = np.concatenate(([0], np.cumsum(lens))).astype(np.int64)
    rows = np.concatenate([np.arange(off[i], off[i + 1]) for i in sel])
    sub_R = int(soff[-1])
    log(f"C-port CPU baseline, {cores} threads, {len(sel)} proteins (every {stride}th)")
    t1 = time.perf_counter()
    otok, _ = O.tokenize_batch(blob, levels, args.df, pos[rows], flags[rows], soff, n_threads=cores)
    cpu_s = time.perf_counter() - t1
    port = {"value": round(sub_R / cpu_s, 1), "unit": "residues/s", "cores": cores, "kind": "port",
            "sample": f"{len(sel)} proteins (every {stride}th of the workload, {sub_R} residues), oracle/pst_oracle.c "
                      f"(ragged, real residues only, the GPU's canonical op order), OpenMP over proteins, {cpu_s:.1f} s"}
    gsel = gpu_tok[rows]
    by_chunk = []
    cuts = plan["cuts"] if plan else [0, nb]
    scheds = plan["schedules"] if plan else [None]
    for c in range(len(cuts) - 1):
        in_c = (sel >= cuts[c]) & (sel < cuts[c + 1])
        r_c = np.concatenate([np.arange(soff[j], soff[j + 1]) for j in np.nonzero(in_c)[0]]) if in_c.any() \
            else np.zeros(0, np.int64)
        by_chunk.append({"proteins": [int(cuts[c]), int(cuts[c + 1])], "schedule": scheds[c],
                         "proteins_compared": int(in_c.sum()), "tokens_compared": int(len(r_c)),
                         "identical": int(np.sum(gsel[r_c] == otok[r_c]))})
    match = int(np.sum(gsel == otok))
    exact = {"tokens_compared": sub_R, "identical": match, "rate": match / sub_R,
             "proteins_compared": int(len(sel)), "sample": f"every {stride}th protein",
             "by_pipeline_chunk": by_chunk,
             "against": "C oracle (bitwise canonical path)"}
    return out[cores], out.get(8), cfg2.get(cores), cfg2.get(8), port, exact


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_workers(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plan:
        return plan_only(args, rank, world)

    import torch
    import torch.distributed as dist
    from pst_amd import params as P
    from pst_amd._native import Tokenizer, pack_samples
    from pst_amd.config import LEVELS

    ndev = max(1, torch.cuda.device_count())
    gpu = local % ndev  # one GPU per rank on a node; ranks share a GPU only when rehearsing with gloo
    if world > 1:
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            init_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            init_group(args.dist_backend)
    dev = torch.device("cuda", gpu)
    red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    seen_world = dist.get_world_size() if world > 1 else 1

    log(f"rank {rank}/{world}: building the synthetic workload")
    ids, samples = workload(args, rank, world)
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    pin_pos = torch.from_numpy(pos).pin_memory()
    pin_flags = torch.from_numpy(flags).pin_memory()
    # the wire format of the timed region: the PDB path's float32 coordinates (pst_tokenize_f32,
    # 481 B per residue) unless --f64-input (pst_tokenize, 925 B); the generator's values are
    # float32-exact, so both give the same tokens (checked below)
    pos32 = pos.astype(np.float32)
    assert np.array_equal(pos32.astype(np.float64), pos), "synthetic coordinates are not float32-exact"
    pin_pos32 = torch.from_numpy(pos32).pin_memory()
    ppos64, pflags = pin_pos.numpy(), pin_flags.numpy()
    ppos = ppos64 if args.f64_input else pin_pos32.numpy()
    levels = LEVELS[args.codebook]
    blob = P.random_blob(len(levels), 1234)
    tk = Tokenizer(gpu, args.codebook, args.df, blob)
    torch.cuda.synchronize(dev)

    # inputs resident in HBM before the timed region (the `value` contract): float64 positions and
    # flags on the device, tokens left in HBM; the host-to-host rate (pinned host atom37 -> H2D ->
    # tokens -> D2H, PCIe included) is measured after it and reported beside it, never as `value`
    d_pos = pin_pos.to(dev)
    d_flags = pin_flags.to(dev)
    d_tok = torch.zeros(R, dtype=torch.int32, device=dev)
    d_ntok = torch.zeros(len(samples), dtype=torch.int32, device=dev)
    d_nn = torch.zeros(len(samples), dtype=torch.int32, device=dev)

    def dstep():
        tk.tokenize_device(d_pos.data_ptr(), d_flags.data_ptr(), off, d_tok.data_ptr(), d_ntok.data_ptr(),
                           d_nn.data_ptr())

    log(f"rank {rank}: {len(samples)} proteins, {R} residues; warm-up")
    for _ in range(args.warmup):
        tk.tokenize_packed(ppos, pflags, off)
        dstep()
        tk.sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # shader clock of the timed steps from libpst's clock counters (pst_clock_counters: stamps of
    # the fused MPNN launches, enabled for the bench only), read once after the timed loop so the
    # bracketed time holds no instrumentation
    tk.set_clock_counters(True)
    tk.clock_counters(reset=True)
    times = []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        t0 = time.perf_counter()
        dstep()  # HBM-resident inputs -> graph -> encoder -> FSQ -> token ids in HBM
        tk.sync()
        times.append(time.perf_counter() - t0)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    clock = clock_stats([tk.clock_counters(reset=True)], steps=args.steps)
    tk.set_clock_counters(False)
    log(f"rank {rank}: {args.steps} timed steps in {elapsed:.2f} s")
    stats = torch.tensor(times + [elapsed], dtype=torch.float64, device=red_dev)
    total_res = torch.tensor([R], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(total_res, op=dist.ReduceOp.SUM)
    stats = stats.cpu().numpy()
    step_s = stats[:-1]
    elapsed = float(stats[-1])
    job_res = int(total_res.item())
    med = float(np.median(step_s))
    value = job_res / med
    dev_tok = d_tok.cpu().numpy().view(np.uint32)

    # host to host (PCIe included): the same steps from pinned host buffers through pst_tokenize_f32
    # (or pst_tokenize with --f64-input), median over as many steps, max over ranks
    h_times = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        tok, nt, nn = tk.tokenize_packed(ppos, pflags, off)  # host -> host, synchronous
        h_times.append(time.perf_counter() - t0)
    plan = tk.last_plan_detail()  # chunks and layer schedule of the host-to-host step (rank 0's share)
    h_stats = torch.tensor([float(np.median(h_times))], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(h_stats, op=dist.ReduceOp.MAX)
    h_med = float(h_stats.cpu().numpy()[0])
    host_to_host = {"residues_per_s": round(job_res / h_med, 1), "ms_per_step": round(h_med * 1e3, 3),
                    "steps": args.steps,
                    "tokens_identical_to_device_resident": bool(np.array_equal(tok[:R], dev_tok[:R])),
                    "note": ("pinned host atom37 -> H2D -> graph -> encoder -> FSQ -> D2H token ids ("
                             + ("pst_tokenize, float64 positions" if args.f64_input else
                                "pst_tokenize_f32, float32 positions as the PDB path holds them")
                             + "), median over steps of the max over ranks; PCIe-inclusive, not `value`")}

    # the other wire format on the same inputs: same tokens, and its host-to-host time (median of 5)
    alt = ppos64 if not args.f64_input else pin_pos32.numpy()
    alt_t = []
    for i in range(6):
        t0 = time.perf_counter()
        tok_alt, _, _ = tk.tokenize_packed(alt, pflags, off)
        if i:
            alt_t.append(time.perf_counter() - t0)
    alt_med = float(np.median(alt_t))
    other_input = {"input": "float64 (pst_tokenize)" if not args.f64_input else "float32 (pst_tokenize_f32)",
                   "residues_per_s_per_gpu": round(R / alt_med, 1), "ms": round(alt_med * 1e3, 3),
                   "tokens_identical": bool(np.array_equal(tok_alt[:R], tok[:R])),
                   "note": "rank 0's shard, host to host, median of 5 after one warm-up"}

    # exact match vs the reference fixtures of the proteins this rank holds (summed over ranks), on
    # the host-to-host step's tokens (identical to the timed device-resident ones, checked above)
    tok, nt, nn = tk.tokenize_packed(ppos, pflags, off)
    ref_match = reference_exact_match(args, ids, tok, off, plan, bounded=tk.aux(R)["bounded"])
    if world > 1:
        cnt = torch.tensor([ref_match["tokens_compared"], ref_match["identical"]] if ref_match else [0, 0],
                           dtype=torch.float64, device=red_dev)
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
        if ref_match:
            ref_match["tokens_compared_all_ranks"] = int(cnt[0].item())
            ref_match["identical_all_ranks"] = int(cnt[1].item())

    # per-stage device times (HIP events on libpst's stream), rank 0's share
    tk.set_clock_counters(True)
    tk.set_timing(True)
    stage = None
    sclk = []
    tk.clock_counters(reset=True)
    for _ in range(3):
        dstep()
        st = tk.stage_ms()
        stage = st if stage is None else {k: stage[k] + st[k] for k in st}
        sclk.append(tk.clock_counters(reset=True))
    stage_clock = clock_stats(sclk)
    # two waves per SIMD (the MPNN kernels' 256 VGPRs), four SIMDs per CU
    occupancy = wave_slot_occupancy(sclk, 8 * torch.cuda.get_device_properties(dev).multi_processor_count)
    stage = {k: v / 3 for k, v in stage.items()}
    tk.set_timing(False)
    tk.set_clock_counters(False)

    kern = {}
    for name in ("mpnn0", "mpnn1", "mpnn2"):
        ms = stage[name]
        ex = MFMA_PER_TASK[name] * MFMA_FLOP * (R / 32) / (ms * 1e-3) / 1e12
        kern[name] = {"launch_ms": round(ms, 3), "executed_mfma_tflops": round(ex, 2),
                      "frac": round(ex / PEAK_FP32_TFLOPS, 4)}
    dom = "mpnn1"
    dom_ms = kern[dom]["launch_ms"]
    executed = kern[dom]["executed_mfma_tflops"]
    traffic = None
    if os.path.exists(args.traffic_file):
        with open(args.traffic_file) as fh:
            tf = json.load(fh)
        per_res = tf["read_bytes_per_residue"] + tf["write_bytes_per_residue"]
        traffic = {"bytes_per_launch": round(per_res * R), "read_bytes_per_residue": tf["read_bytes_per_residue"],
                   "write_bytes_per_residue": tf["write_bytes_per_residue"],
                   "achieved_GBps": round(per_res * R / (dom_ms * 1e-3) / 1e9, 1),
                   "source": tf.get("source", args.traffic_file)}
    roofline = {
        "kernel": "k_mpnn<1> (edge MLP L1 + message MLP L2 + node FFN, fused)",
        "bound": "mfma", "achieved": executed, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
        "frac": round(executed / PEAK_FP32_TFLOPS, 4),
        "traffic": traffic["bytes_per_launch"] if traffic else None,  # HBM bytes per launch (PMC)
        "traffic_detail": traffic,
        "note": "achieved = executed v_mfma_f32_32x32x2_f32 FLOPs per launch (MFMA_PER_TASK, = PMC "
                "SQ_INSTS_MFMA) / HIP-event launch time; effective_alg_tflops counts SURVEY 8d's algorithmic "
                "FLOPs instead, which the kernel's algebraic rewrites (DESIGN.md 5) execute in 0.52x the work",
        "launch_ms": round(dom_ms, 3),
        "effective_alg_tflops": round(MPNN1_ALG_FLOP_PER_RES * R / (dom_ms * 1e-3) / 1e12, 2),
        # the peak is quoted at the 2.4 GHz spec clock; at the clock the chip actually held under
        # k_mpnn<1> in the stage-timing steps (its launches' clock stamps) the reachable peak is
        # peak x clock / 2.4
        "stage_clock": stage_clock,
        "frac_at_measured_clock": (round(executed / (PEAK_FP32_TFLOPS * stage_clock["per_layer_ghz"][1] / SPEC_GHZ), 4)
                                   if stage_clock else None),
        "wave_slot_occupancy": occupancy,
        "kernels": kern,
        "stage_ms": {k: round(v, 3) for k, v in stage.items()},
        "path_effective_alg_tflops": (round(PATH_ALG_FLOP_PER_RES[args.df] * R / (sum(stage.values()) * 1e-3) / 1e12, 2)
                                      if args.df in PATH_ALG_FLOP_PER_RES else None),
    }

    log("device-resident rate and stage times done")
    e2e, casp = casp14_end_to_end(tk) if (rank == 0 and world == 1 and not args.no_e2e) else (None, None)
    cpu = cpu8 = cpu_c2 = cpu_c2_8 = port = exact = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("CPU baselines")
        cpu, cpu8, cpu_c2, cpu_c2_8, port, exact = cpu_baselines(args, samples, blob, levels, pos, flags, off, tok,
                                                                 plan, casp, ref_ids=ids)

    if rank == 0:
        mode = "weak" if args.weak else "strong"
        out = {
            "metric": f"residues tokenized/sec (cb={args.codebook}, df={args.df})",
            "value": round(value, 1),
            "unit": "residues/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(med * 1e3, 3),
            "higher_is_better": True,
            "scaling": mode,
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (random-walk backbones, seeds 1000+p; random-init weights of the reference architecture)",
            "config": {"workload": (f"{args.proteins} proteins x {args.residues} residues "
                                    f"{'per GPU' if args.weak else 'per job, batch-sharded over the GPUs'}, "
                                    f"codebook {args.codebook}, df {args.df}"),
                       "codebook_size": args.codebook, "df": args.df, "residues_per_protein": args.residues,
                       "proteins_job": args.proteins * (world if args.weak else 1), "residues_job": job_res,
                       "proteins_rank0": len(ids), "parallelism": f"dp{world} (independent proteins, LPT shard)",
                       "world_size_seen": seen_world, "dist_backend": args.dist_backend if world > 1 else None},
            "timed_region": ("atom37 (float64) + flags already resident in HBM -> graph -> encoder -> FSQ -> token "
                             "ids in HBM (pst_tokenize_device, synchronised per step), median over steps of the "
                             "max over ranks"),
            "host_to_host": host_to_host,
            "other_input_format": other_input,
            "pipeline_plan": plan,
            "ms_per_step_mean_bracketed": round(elapsed / args.steps * 1e3, 3),
            "elapsed_s": round(elapsed, 3),
            "clock": clock,
            "ms_per_step_at_2p4ghz": (round(med * 1e3 * clock["mean_ghz"] / SPEC_GHZ, 3) if clock else None),
            "clock_note": ("shader clock of the timed steps (rank 0): s_memtime / s_memrealtime stamps of the "
                           "fused MPNN launches (pst_clock_counters), per step over its three layers; "
                           "ms_per_step_at_2p4ghz scales the median step by mean_ghz / 2.4 as if all of it "
                           "were clock-bound"),
            "roofline": roofline,
            "exact_match_reference": ref_match,
            "exact_match": exact,
            "cpu_baseline": cpu,
            "cpu_baseline_8_threads": cpu8,
            "cpu_baseline_config2": cpu_c2,
            "cpu_baseline_config2_8_threads": cpu_c2_8,
            "cpu_baseline_ragged_port": port,
            "casp14_end_to_end": e2e,
        }
        try:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            from provenance import provenance
            out["provenance"] = provenance()
        except Exception as ex:  # measurement metadata only
            out["provenance"] = {"error": str(ex)}
        print(json.dumps(out), flush=True)
    tk.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
