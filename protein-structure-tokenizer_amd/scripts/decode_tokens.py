"""Decode token files back to backbone structures — drop-in for the reference's
`scripts/decode_tokens.py` (same flags; `--backend gpu` only; `--weights_dir` / `--config_path`
added). Writes `<structure_save_path>/structures/structure_<stem>.pdb` for every
`<stem>_tokens.npy` in `--tokens_dir` (scripts/inference_runner.py:326-437).
"""
import argparse
import os
import sys
from typing import List, Optional

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from pst_amd import config as C  # noqa: E402
from pst_amd.runner import InferenceRunner  # noqa: E402


def main(sequences: List[str], structure_save_path: str, backend: str, batch_size_per_device: int = 8,
         config_overrides: Optional[List[str]] = None, *, weights_dir: Optional[str] = None,
         config_path: Optional[str] = None):
    """The reference's `main` (`scripts/decode_tokens.py:32-80`), same positional signature; the
    model comes from `config_overrides` as in `tokenize_pdb.main`
    (`pst_amd.config.config_from_overrides`). Keyword-only extras: `weights_dir`, `config_path`."""
    if config_path:
        cfg = C.config_from_hydra(C.load_config("vq3d_inference", job_name="tokenize",
                                                overrides=config_overrides, config_path=config_path))
    else:
        cfg = C.config_from_overrides(config_overrides)
    runner = InferenceRunner()
    local_devices, n_local_device = runner.prepare_devices(backend=backend)
    decode_fn = runner.prepare_decode_fn(cfg=cfg, devices=local_devices)
    indexes_to_codes_fn = runner.prepare_token_to_code_fn(cfg=cfg, devices=local_devices)
    model_params = runner.load_params(model_dir=weights_dir or cfg.weight_dir, local_devices=local_devices)
    try:
        runner.decode_and_save_pdbs(random_key=None, decode=decode_fn, indexes_to_codes_fn=indexes_to_codes_fn,
                                    sequences=sequences, model_params=model_params, num_device=n_local_device,
                                    structure_save_path=structure_save_path,
                                    batch_size_per_device=batch_size_per_device, max_seq_len=cfg.seq_max_size,
                                    downsampling_ratio=cfg.downsampling_ratio, pad_token_id=cfg.pad_token_id)
    finally:
        decode_fn.close()


def cli(argv=None):
    parser = argparse.ArgumentParser(description="Tokenizer specification !")
    parser.add_argument("--model_downsampling", type=int, choices=[1, 2, 4], default=1)
    parser.add_argument("--codebook_size", type=int, choices=[432, 1728, 4096, 64000], default=4096)
    parser.add_argument("--structure_save_path", type=str, required=True)
    parser.add_argument("--tokens_dir", type=str, required=True, help="folder containing the *_tokens.npy files")
    parser.add_argument("--backend", type=str, default="gpu", choices=["gpu", "tpu", "cpu"])
    parser.add_argument("--batch_size_per_device", type=int, default=1)
    parser.add_argument("--weights_dir", type=str, default=None)
    parser.add_argument("--config_path", type=str, default=None)
    args = parser.parse_args(argv)
    df = args.model_downsampling
    if (args.codebook_size, df) not in C.SHIPPED:
        raise SystemExit(f"no model for codebook_size={args.codebook_size}, df={df}")
    tokens = [os.path.join(args.tokens_dir, f) for f in os.listdir(args.tokens_dir)]
    main(sequences=tokens, structure_save_path=args.structure_save_path, backend=args.backend,
         batch_size_per_device=args.batch_size_per_device, weights_dir=args.weights_dir,
         config_path=args.config_path, config_overrides=C.overrides_for(args.codebook_size, df))


if __name__ == "__main__":
    cli()
