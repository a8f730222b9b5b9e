"""The collectives bench.py issues under torchrun with the nccl (= RCCL) backend, exercised on a
one-GPU box as a world of one: init with device_id, barrier, float64 all_reduce MAX / SUM on the
device. Prints one JSON line.

    python tools/nccl_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "protein-structure-tokenizer_amd")]
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bench import init_group  # noqa: E402


def main():
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    init_group("nccl", device_id=torch.device("cuda", 0))
    t_init = time.perf_counter() - t0
    dist.barrier()
    stats = torch.tensor([0.05, 0.06, 1.1], dtype=torch.float64, device="cuda")
    total = torch.tensor([262144.0], dtype=torch.float64, device="cuda")
    dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    dist.all_reduce(total, op=dist.ReduceOp.SUM)
    torch.cuda.synchronize()
    out = {"backend": dist.get_backend(), "world": dist.get_world_size(), "init_s": round(t_init, 3),
           "max": stats.cpu().tolist(), "sum": total.cpu().tolist(),
           "nccl_version": ".".join(map(str, torch.cuda.nccl.version()))}
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
