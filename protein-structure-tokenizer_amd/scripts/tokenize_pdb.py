"""Tokenize a directory of PDB files — drop-in for the reference's `scripts/tokenize_pdb.py`.

    python protein-structure-tokenizer_amd/scripts/tokenize_pdb.py \\
        --pdb_dir DIR --token_save_path OUT [--codebook_size 4096] [--model_downsampling 1] \\
        [--batch_size_per_device 1] [--weights_dir weights/4k_df_1/] [--config_path CFG]

Same arguments and outputs (`OUT/<pdb stem>_tokens.npy`, uint32 [1, n_tokens]) as the
reference (`scripts/tokenize_pdb.py:79-121`); `--backend` accepts only "gpu" (the default
here). The model directory must hold `params.npz` (read with `allow_pickle=False`; the pickled
`state_variables.npy` is not needed). The CLI builds the reference's two overrides from its
flags (`model=gnn/ablation_<K>_df_<df>.yaml`, `data=ablation_df_<df>.yaml`) and `main` selects
the model from them (`pst_amd.config.config_from_overrides`, no YAML tree needed); with
`--config_path` the reference's YAML tree is composed from the same overrides instead.
The reference's CLI defaults `--backend` to "cpu" (an XLA target); libpst has no CPU path, so
the default here is "gpu" and any other backend raises NotImplementedError.

One process drives every local GPU (a host thread per GPU, like the reference's pmap). Under
`torchrun` (WORLD_SIZE > 1) each rank instead takes GPU LOCAL_RANK (modulo the visible devices)
and an LPT shard of the PDB list balanced on file size (`runner.shard_for_rank`); there is no
collective on the data path. Rank 0 creates `--token_save_path` exactly as the reference does
(`inference_runner.py:265`, FileExistsError if it exists; any other OSError is re-raised on
every rank with its type) and broadcasts the outcome over a gloo group before any rank starts;
each rank writes through a private `.rank<N>` directory inside it.
"""
import argparse
import os
import sys
from typing import List, Optional

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from pst_amd import config as C  # noqa: E402
from pst_amd.runner import InferenceRunner, shard_for_rank  # noqa: E402


def main(pdbs: List[str], token_save_path: str, backend: str, batch_size_per_device: int = 8,
         config_name: Optional[str] = None, config_overrides: Optional[List[str]] = None, *,
         weights_dir: Optional[str] = None, config_path: Optional[str] = None):
    """The reference's `main` (`scripts/tokenize_pdb.py:32-73`), same positional signature.

    The model is selected by `config_overrides` exactly as the reference composes it
    (`model=gnn/ablation_<K>_df_<df>.yaml`, `data=ablation_df_<df>.yaml`,
    `pst_amd.config.config_from_overrides`); an unrecognised override raises instead of
    falling back to a default. `config_name` is accepted and, as in the reference, not used:
    the composed config is always `vq3d_inference` (`/root/reference/scripts/tokenize_pdb.py:40-45`),
    also when `config_path` points at the reference's YAML tree, which is then composed with
    Hydra's rules.
    Keyword-only extras: `weights_dir` (directory of `params.npz`; default the config's
    `weight_paths`) and `config_path`.
    """
    if config_path:
        cfg = C.config_from_hydra(C.load_config("vq3d_inference", job_name="tokenize",
                                                overrides=config_overrides, config_path=config_path))
    else:
        cfg = C.config_from_overrides(config_overrides)
    runner = InferenceRunner()
    local_devices, n_local_device = runner.prepare_devices(backend=backend)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        rank = int(os.environ.get("RANK", "0"))
        _create_output_on_rank0(token_save_path, rank)
        local_devices = [int(os.environ.get("LOCAL_RANK", "0")) % n_local_device]
        # LPT on PDB text size (∝ atoms ∝ residues) balances residues per GPU
        pdbs = sorted(pdbs)
        pdbs = shard_for_rank(pdbs, rank, world, weights=[os.path.getsize(p) for p in pdbs])
        if not pdbs:
            return
    tokenize = runner.prepare_tokenize_fn(cfg=cfg, devices=local_devices)
    model_params = runner.load_params(model_dir=weights_dir or cfg.weight_dir, local_devices=local_devices)
    try:
        if world > 1:
            _tokenize_rank(runner, tokenize, model_params, pdbs, token_save_path, cfg, batch_size_per_device)
        else:
            runner.tokenize(random_key=None, quantize=tokenize, model_params=model_params, pdbs=pdbs,
                            token_save_path=token_save_path, num_device=len(local_devices),
                            data_config=cfg, batch_size_per_device=batch_size_per_device)
    finally:
        tokenize.close()


def _create_output_on_rank0(token_save_path: str, rank: int) -> None:
    """`os.makedirs(token_save_path, exist_ok=False)` once for the job (inference_runner.py:265):
    rank 0 creates it, every rank raises the same FileExistsError if it already existed."""
    import torch.distributed as dist
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo")  # env:// from torchrun; control only, no data
    try:
        msg = [None]
        if rank == 0:
            # any failure (exists, permission, bad parent...) must reach every rank before the
            # broadcast, or the other ranks would wait in it until the gloo timeout
            try:
                os.makedirs(token_save_path, exist_ok=False)
            except OSError as e:
                msg = [(type(e).__name__, e.errno, e.strerror, e.filename)]
            except Exception as e:  # noqa: BLE001 — e.g. a TypeError from a bad path object
                msg = [("RuntimeError", None, f"{type(e).__name__}: {e}", None)]
        dist.broadcast_object_list(msg, src=0)
        if msg[0] is not None:
            name, errno_, strerror, filename = msg[0]
            if name == "RuntimeError":
                raise RuntimeError(strerror)
            exc = {"FileExistsError": FileExistsError, "PermissionError": PermissionError,
                   "FileNotFoundError": FileNotFoundError, "NotADirectoryError": NotADirectoryError
                   }.get(name, OSError)
            raise exc(errno_, strerror, filename)
    finally:
        if own:
            dist.destroy_process_group()


def _tokenize_rank(runner, tokenize, model_params, pdbs, token_save_path, cfg, bs):
    # every rank writes into the directory rank 0 created; rank files are disjoint by construction
    tmp = os.path.join(token_save_path, f".rank{os.environ.get('RANK', '0')}")
    runner.tokenize(random_key=None, quantize=tokenize, model_params=model_params, pdbs=pdbs,
                    token_save_path=tmp, num_device=1, data_config=cfg, batch_size_per_device=bs)
    for f in os.listdir(tmp):
        os.replace(os.path.join(tmp, f), os.path.join(token_save_path, f))
    os.rmdir(tmp)


def cli(argv=None):
    parser = argparse.ArgumentParser(description="Tokenizer specification !")
    parser.add_argument("--model_downsampling", type=int, choices=[1, 2, 4], default=1)
    parser.add_argument("--codebook_size", type=int, choices=[432, 1728, 4096, 64000], default=4096)
    parser.add_argument("--token_save_path", type=str, required=True)
    parser.add_argument("--pdb_dir", type=str, required=True, help="folder containing the .pdb files to be tokenized")
    parser.add_argument("--backend", type=str, default="gpu", choices=["gpu", "tpu", "cpu"])
    parser.add_argument("--batch_size_per_device", type=int, default=1)
    parser.add_argument("--weights_dir", type=str, default=None,
                        help="model directory holding params.npz (default: the config's weight_paths)")
    parser.add_argument("--config_path", type=str, default=None,
                        help="the reference's config/structure_tokenizer tree (optional)")
    args = parser.parse_args(argv)
    df = args.model_downsampling
    if (args.codebook_size, df) not in C.SHIPPED:
        raise SystemExit(f"no model for codebook_size={args.codebook_size}, df={df}")
    pdbs = [os.path.join(args.pdb_dir, f) for f in os.listdir(args.pdb_dir)]
    main(pdbs=pdbs, token_save_path=args.token_save_path, backend=args.backend,
         batch_size_per_device=args.batch_size_per_device, weights_dir=args.weights_dir,
         config_path=args.config_path, config_overrides=C.overrides_for(args.codebook_size, df))


if __name__ == "__main__":
    cli()
