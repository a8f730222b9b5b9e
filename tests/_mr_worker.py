"""Worker for test_multirank.py (one process per rank, gloo on 127.0.0.1)."""
import os
import sys


def run(rank, world, port, pdb_dir, model_dir, out_dir, result_q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (root, os.path.join(root, "protein-structure-tokenizer_amd"), here):
        sys.path.insert(0, p)
    import numpy as np
    import torch.distributed as dist
    from pst_amd import runner
    from test_host import OracleTokenizeFn

    sys.path.insert(0, os.path.join(root, "protein-structure-tokenizer_amd", "scripts"))
    import tokenize_pdb as cli

    # the per-GPU device query and compute are swapped for the CPU oracle; the CLI's rank
    # sharding, file handling and runner loop are the product code
    runner.InferenceRunner.prepare_devices = staticmethod(lambda backend="gpu": ([0], 1))
    runner.InferenceRunner.prepare_tokenize_fn = staticmethod(lambda cfg, devices: OracleTokenizeFn(cfg, devices))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pdbs = [os.path.join(pdb_dir, f) for f in os.listdir(pdb_dir)]
    pdbs_sorted = sorted(pdbs)
    mine = runner.shard_for_rank(pdbs_sorted, rank, world, weights=[os.path.getsize(p) for p in pdbs_sorted])
    cli.main(pdbs=pdbs, token_save_path=out_dir, backend="gpu", batch_size_per_device=2,
             config_overrides=["model=gnn/ablation_4k_df_1.yaml", "data=ablation_df_1.yaml"], weights_dir=model_dir)
    # host-side gather of what each rank handled (test bookkeeping only, not the data path)
    got = [None] * world
    dist.all_gather_object(got, sorted(os.path.basename(p) for p in mine))
    dist.barrier()
    if rank == 0:
        result_q.put(got)
    dist.destroy_process_group()


def run_ppl(rank, world, port, hists, result_q):
    """global_perplexity over `world` gloo ranks, rank r holding hists[r]."""
    import torch.distributed as dist
    from pst_amd import runner
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    v = runner.global_perplexity(hists[rank])
    got = [None] * world
    dist.all_gather_object(got, v)
    if rank == 0:
        result_q.put(got)
    dist.destroy_process_group()


def run_existing_dir(rank, world, port, pdb_dir, model_dir, out_dir, result_q):
    """Both ranks must raise FileExistsError when the output directory already exists
    (rank 0 decides, inference_runner.py:265), and nothing may be written into it."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (root, os.path.join(root, "protein-structure-tokenizer_amd"), here,
              os.path.join(root, "protein-structure-tokenizer_amd", "scripts")):
        sys.path.insert(0, p)
    from pst_amd import runner
    from test_host import OracleTokenizeFn
    import tokenize_pdb as cli
    runner.InferenceRunner.prepare_devices = staticmethod(lambda backend="gpu": ([0], 1))
    runner.InferenceRunner.prepare_tokenize_fn = staticmethod(lambda cfg, devices: OracleTokenizeFn(cfg, devices))
    pdbs = [os.path.join(pdb_dir, f) for f in os.listdir(pdb_dir)]
    try:
        cli.main(pdbs=pdbs, token_save_path=out_dir, backend="gpu", batch_size_per_device=2,
                 config_overrides=["model=gnn/ablation_4k_df_1.yaml", "data=ablation_df_1.yaml"], weights_dir=model_dir)
        result_q.put((rank, "no error"))
    except FileExistsError:
        result_q.put((rank, "FileExistsError"))
