"""Benchmark: residues tokenized/s (codebook 4096, df 1) on MI355X — BASELINE.json's metric.

One step = one pass of the tokenize hot path (graph build → 3 fused MPNN layers →
downsampler → FSQ ids) over one batch of 1024 synthetic proteins x 256 residues per GPU, with
the atom37 inputs already resident in HBM (pst_tokenize_device). Multi-GPU: one process per
GPU (torchrun), independent proteins per rank, no collective on the data path ("scaling":
"weak": every rank runs the full 1024 x 256 workload on its own proteins). Prints ONE JSON line
on rank 0.

Also reported: the dominant kernel's roofline (HIP events on the library's stream), the CPU
baseline (the oracle, C, on a bounded sample on this host's cores) and the GPU-vs-oracle token
exact-match rate on that sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pst_amd import params as P  # noqa: E402
from pst_amd import synthetic  # noqa: E402
from pst_amd._native import Tokenizer, pack_samples  # noqa: E402

N_PROT, N_RES, CODEBOOK, DF = 1024, 256, 4096, 1
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32 MFMA / VALU dense peak
PEAK_HBM_GBS = 8000.0
H, K = 128, 50
# Algorithmic FLOPs (padding and dead code removed) of the dominant kernel
# k_mpnn<1> = edge MLP of layer 1 + message MLP of layer 2 over 50 edges, + layer-2 node FFN:
MLP_FLOP = 2 * (3 * H * H + H * H + H * H)          # 163 840 per edge per 384-128-128-128 MLP
MPNN1_ALG_FLOP_PER_RES = K * 2 * MLP_FLOP + 2 * (H * 4 * H + 4 * H * H)   # 16 646 144
PATH_ALG_FLOP_PER_RES = {1: 44_715_008, 4: 44_395_904}  # SURVEY §8d, whole path per residue
# What k_mpnn<1> executes: node-projection split of the 384-wide first layers
# (edge MLP 3 GEMMs of 128x128 per edge, message MLP 2 per edge), the message MLP's last layer
# once per receiver after the segment sum, the 4 node projections and the node FFN
MPNN1_EXEC_FLOP_PER_RES = K * 5 * 2 * H * H + 2 * H * H + 4 * 2 * H * H + 2 * (H * 4 * H + 4 * H * H)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--proteins", type=int, default=N_PROT)
    ap.add_argument("--residues", type=int, default=N_RES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the CASP14 end-to-end field")
    ap.add_argument("--codebook", type=int, default=CODEBOOK, help="secondary configs (default: the metric's 4096)")
    ap.add_argument("--df", type=int, default=DF)
    ap.add_argument("--cpu-sample", type=int, default=256, help="proteins in the CPU-baseline sample")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_k_mpnn1.json"),
                    help="PMC-measured HBM bytes per residue of k_mpnn<1> (tools/pmc_traffic.sh)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, the driver's runs) or gloo (rehearsing several ranks on one GPU)")
    return ap.parse_args()


def casp14_end_to_end(tk):
    """SURVEY config 2 as the CLI runs it: parse the 31 CASP14 PDB files (native parser, 16
    threads), tokenize from host buffers, write <stem>_tokens.npy. Reported beside `value`."""
    import tarfile
    import tempfile
    from pst_amd._native import parse_pdb_files
    arc = os.path.join(ROOT, "tests", "golden", "casp14_pdbs.tar.gz")
    if not os.path.exists(arc):
        return None
    with tempfile.TemporaryDirectory() as d:
        with tarfile.open(arc) as tf:
            tf.extractall(d, members=[m for m in tf.getmembers() if m.isfile() and m.name.endswith(".pdb")])
        files = sorted(os.path.join(d, "casp14_pdbs", f) for f in os.listdir(os.path.join(d, "casp14_pdbs")))
        os.makedirs(os.path.join(d, "out"))
        t0 = time.perf_counter()
        B = parse_pdb_files(files, n_threads=16)
        t1 = time.perf_counter()
        tok, nt, _ = tk.tokenize_packed(B.positions, B.flags, B.offsets)
        t2 = time.perf_counter()
        for i, f in enumerate(files):
            a = int(B.offsets[i])
            np.save(os.path.join(d, "out", os.path.basename(f)[:-4] + "_tokens"), tok[a:a + nt[i]].reshape(1, -1))
        t3 = time.perf_counter()
    R = int(B.offsets[-1])
    return {"workload": "CASP14 31 structures (SURVEY config 2), codebook 4096, df 1", "residues": R,
            "parse_ms": round((t1 - t0) * 1e3, 2), "tokenize_ms": round((t2 - t1) * 1e3, 2),
            "write_ms": round((t3 - t2) * 1e3, 2), "residues_per_s": round(R / (t3 - t0), 1)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    gpu = local % ndev  # one GPU per rank on a full node; ranks share GPUs only when rehearsing with gloo
    if world > 1:
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", gpu)
    red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    # synthetic workload of this rank (different proteins per rank)
    samples = synthetic.synthetic_batch(args.proteins, args.residues, seed=1000 + rank * 100_000)
    pos, flags, off = pack_samples(samples)
    d_pos = torch.from_numpy(pos).to(dev)
    d_flags = torch.from_numpy(flags).to(dev)
    R = int(off[-1])
    d_tok = torch.zeros(R, dtype=torch.int32, device=dev)
    d_ntok = torch.zeros(len(samples), dtype=torch.int32, device=dev)
    d_nn = torch.zeros(len(samples), dtype=torch.int32, device=dev)
    from pst_amd.config import LEVELS
    levels = LEVELS[args.codebook]
    blob = P.random_blob(len(levels), 1234)
    tk = Tokenizer(gpu, args.codebook, args.df, blob)
    torch.cuda.synchronize(dev)

    def step():
        tk.tokenize_device(d_pos.data_ptr(), d_flags.data_ptr(), off, d_tok.data_ptr(), d_ntok.data_ptr(),
                           d_nn.data_ptr())

    for _ in range(args.warmup):
        step()
    tk.sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    tk.sync()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    residues_per_rank = R
    value = world * residues_per_rank * args.steps / elapsed

    # per-stage device times (HIP events on the library stream), averaged over 3 extra steps
    tk.set_timing(True)
    stage = None
    for _ in range(3):
        step()
        st = tk.stage_ms()
        stage = st if stage is None else {k: stage[k] + st[k] for k in st}
    stage = {k: v / 3 for k, v in stage.items()}
    tk.set_timing(False)
    dom_ms = stage["mpnn1"]
    achieved = MPNN1_ALG_FLOP_PER_RES * residues_per_rank / (dom_ms * 1e-3) / 1e12
    executed = MPNN1_EXEC_FLOP_PER_RES * residues_per_rank / (dom_ms * 1e-3) / 1e12
    traffic = None
    if os.path.exists(args.traffic_file):
        with open(args.traffic_file) as fh:
            tf = json.load(fh)
        traffic = {"bytes_per_launch": round((tf["read_bytes_per_residue"] + tf["write_bytes_per_residue"])
                                             * residues_per_rank),
                   "read_bytes_per_residue": tf["read_bytes_per_residue"],
                   "write_bytes_per_residue": tf["write_bytes_per_residue"],
                   "achieved_GBps": round((tf["read_bytes_per_residue"] + tf["write_bytes_per_residue"])
                                          * residues_per_rank / (dom_ms * 1e-3) / 1e9, 1),
                   "source": tf.get("source", args.traffic_file)}
    roofline = {
        "kernel": "k_mpnn<1> (edge MLP L1 + message MLP L2 + node FFN, fused)",
        "bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
        "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
        "traffic": traffic["bytes_per_launch"] if traffic else None,  # HBM bytes per launch (PMC)
        "traffic_detail": traffic,
        "note": "achieved/frac count SURVEY 8d algorithmic FLOPs; the kernel executes "
                f"{MPNN1_EXEC_FLOP_PER_RES / MPNN1_ALG_FLOP_PER_RES:.3f}x of them (node-projection split, "
                "message last layer after the segment sum; DESIGN.md 5): executed_tflops/peak = frac_executed",
        "launch_ms": round(dom_ms, 3),
        "executed_tflops": round(executed, 2),
        "frac_executed": round(executed / PEAK_FP32_TFLOPS, 4),
        "stage_ms": {k: round(v, 3) for k, v in stage.items()},
        "path_alg_tflops": (round(PATH_ALG_FLOP_PER_RES[args.df] * residues_per_rank / (sum(stage.values()) * 1e-3) / 1e12, 2)
                            if args.df in PATH_ALG_FLOP_PER_RES else None),
    }

    # PCIe-inclusive rate: host buffers in, host token ids out (pst_tokenize); never `value`
    t2 = time.perf_counter()
    tk.tokenize_packed(pos, flags, off)
    pcie_rate = residues_per_rank / (time.perf_counter() - t2)

    e2e = casp14_end_to_end(tk) if (rank == 0 and world == 1 and not args.no_e2e) else None

    cpu = None
    exact = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        n = min(args.cpu_sample, len(samples))
        sub_off = off[:n + 1]
        sub_R = int(sub_off[-1])
        t1 = time.perf_counter()
        otok, ont = O.tokenize_batch(blob, levels, args.df, pos[:sub_R], flags[:sub_R], sub_off, n_threads=args.cpu_threads)
        cpu_s = time.perf_counter() - t1
        cpu = {"value": round(sub_R / cpu_s, 1), "unit": "residues/s", "cores": args.cpu_threads, "kind": "port",
               "sample": f"first {n} of the synthetic proteins ({sub_R} residues), oracle/pst_oracle.c, "
                         f"OpenMP over proteins, {cpu_s:.1f} s"}
        gtok = d_tok.cpu().numpy().view(np.uint32)
        match = int(np.sum(gtok[:sub_R] == otok[:sub_R]))
        exact = {"tokens_compared": sub_R, "identical": match, "rate": match / sub_R, "against": "oracle (bitwise canonical path)"}

    if rank == 0:
        out = {
            "metric": f"residues tokenized/sec (cb={args.codebook}, df={args.df})",
            "value": round(value, 1),
            "unit": "residues/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (random-walk backbones, random-init weights of the reference architecture)",
            "config": {"workload": f"{args.proteins} proteins x {args.residues} residues per GPU, codebook {args.codebook}, df {args.df}",
                       "codebook_size": args.codebook, "df": args.df, "proteins_per_gpu": args.proteins,
                       "residues_per_protein": args.residues, "parallelism": f"dp{world} (independent proteins)"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "exact_match": exact,
            "pcie_inclusive_residues_per_s_per_gpu": round(pcie_rate, 1),
            "casp14_end_to_end": e2e,
        }
        print(json.dumps(out), flush=True)
    tk.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
