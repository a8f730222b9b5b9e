"""Encoder-half parameters: haiku names, shapes, the flat blob the C ABI takes, random init.

Names are the haiku paths the reference creates for `Vq3D.encode_and_quantize` after
`params_keys_conversion` strips `forward_vq3_d/` (`scripts/inference_runner.py:153-165`);
`tests/test_golden_host.py` checks them against the reference model initialised under the
test shim. The blob is every tensor below, row-major, concatenated in `param_spec` order — the
layout `include/pst.h` documents (`pst_param_count`).
"""
import os
from typing import Dict, List, Tuple

import numpy as np

H = 128
ENC = "vq3_d/~/structure_encoder"
GNN = ENC + "/~/graph_neural_network/~/mpnn_layer"
DS = "vq3_d/~/cross_attn_downsampling/cross_attn_scaler_iteration"


def _layer(l: int) -> str:
    return GNN + ("" if l == 0 else f"_{l}")


def param_spec(codes_dim: int = 6, n_block: int = 3, n_layer: int = 3) -> List[Tuple[str, str, Tuple[int, ...]]]:
    s: List[Tuple[str, str, Tuple[int, ...]]] = []
    s += [(ENC + "/init_node_embed", "w", (H, H)), (ENC + "/init_node_embed", "b", (H,))]
    s += [(ENC + "/init_edge_embed", "w", (H + 27, H)), (ENC + "/init_edge_embed", "b", (H,))]
    for l in range(n_layer):
        p = _layer(l)
        for mlp in ("node_mlp_0",):
            for i, (fi, fo) in enumerate(((3 * H, H), (H, H), (H, H))):
                s += [(f"{p}/{mlp}/~/linear_{i}", "w", (fi, fo)), (f"{p}/{mlp}/~/linear_{i}", "b", (fo,))]
        for i, (fi, fo) in enumerate(((H, 4 * H), (4 * H, H))):
            s += [(f"{p}/node_mlp_1/~/linear_{i}", "w", (fi, fo)), (f"{p}/node_mlp_1/~/linear_{i}", "b", (fo,))]
        for i, (fi, fo) in enumerate(((3 * H, H), (H, H), (H, H))):
            s += [(f"{p}/edge_mlp/~/linear_{i}", "w", (fi, fo)), (f"{p}/edge_mlp/~/linear_{i}", "b", (fo,))]
        for nm in ("norm_msg", "norm_msg_1", "norm_msg_2"):
            s += [(f"{p}/{nm}", "scale", (H,)), (f"{p}/{nm}", "offset", (H,))]
    B = n_block
    for nm in ("query_norm", "data_norm"):
        s += [(f"{DS}/cross_attention/{nm}", "scale", (B, H)), (f"{DS}/cross_attention/{nm}", "offset", (B, H))]
    att = f"{DS}/cross_attention/attention"
    for w in ("query_w", "key_w", "value_w", "gating_w"):
        s += [(att, w, (B, H, 4, 32))]
    s += [(att, "gating_b", (B, 4, 32)), (att, "output_w", (B, 4, 32, H)), (att, "output_b", (B, H))]
    for tr in ("resampled_transition", "original_transition"):
        s += [(f"{DS}/{tr}/input_layer_norm", "scale", (B, H)), (f"{DS}/{tr}/input_layer_norm", "offset", (B, H))]
        s += [(f"{DS}/{tr}/transition1", "weights", (B, H, 2 * H)), (f"{DS}/{tr}/transition1", "bias", (B, 2 * H))]
        s += [(f"{DS}/{tr}/transition2", "weights", (B, 2 * H, H)), (f"{DS}/{tr}/transition2", "bias", (B, H))]
    s += [("vq3_d/down_proj", "w", (H, codes_dim)), ("vq3_d/down_proj", "b", (codes_dim,))]
    return s


def param_count(codes_dim: int = 6) -> int:
    return int(sum(np.prod(sh) for _, _, sh in param_spec(codes_dim)))


def pack(params: Dict[str, Dict[str, np.ndarray]], codes_dim: int = 6) -> np.ndarray:
    """haiku-style nested dict → contiguous float32 blob in `param_spec` order."""
    parts = []
    for mod, name, shape in param_spec(codes_dim):
        try:
            a = np.asarray(params[mod][name], dtype=np.float32)
        except KeyError as e:
            raise KeyError(f"missing parameter {mod}/{name}") from e
        if a.shape != shape:
            raise ValueError(f"{mod}/{name}: expected shape {shape}, got {a.shape}")
        parts.append(a.reshape(-1))
    return np.ascontiguousarray(np.concatenate(parts))


def unpack(blob: np.ndarray, codes_dim: int = 6) -> Dict[str, Dict[str, np.ndarray]]:
    out: Dict[str, Dict[str, np.ndarray]] = {}
    o = 0
    for mod, name, shape in param_spec(codes_dim):
        n = int(np.prod(shape))
        out.setdefault(mod, {})[name] = blob[o:o + n].reshape(shape)
        o += n
    return out


def random_params(codes_dim: int = 6, seed: int = 0, z_scale: float = 1.5) -> Dict[str, Dict[str, np.ndarray]]:
    """Random-init weights of the reference architecture (no checkpoint is available offline).

    Weights: truncated normal (±2σ) with σ = 1/sqrt(fan_in) (haiku fan-in VarianceScaling);
    biases / LayerNorm offsets N(0, 0.1²); LayerNorm scales 1 + N(0, 0.1²); gating bias
    1 + N(0, 0.1²). `down_proj` uses σ = z_scale (its input is unit-norm) so the FSQ latents
    spread over all code levels and the token ids are diverse.
    """
    rng = np.random.default_rng(seed)
    out: Dict[str, Dict[str, np.ndarray]] = {}
    for mod, name, shape in param_spec(codes_dim):
        stacked = mod.startswith(DS)
        core = shape[1:] if stacked else shape
        if name in ("w", "weights", "query_w", "key_w", "value_w", "gating_w", "output_w"):
            if mod == "vq3_d/down_proj":
                sd = z_scale
            elif name == "output_w":
                sd = 1.0 / np.sqrt(core[0] * core[1])
            else:
                sd = 1.0 / np.sqrt(core[0])
            v = np.clip(rng.standard_normal(shape), -2, 2) * sd
        elif name == "scale":
            v = 1.0 + 0.1 * rng.standard_normal(shape)
        elif name == "gating_b":
            v = 1.0 + 0.1 * rng.standard_normal(shape)
        else:  # b, bias, offset, output_b
            v = 0.1 * rng.standard_normal(shape)
        out.setdefault(mod, {})[name] = v.astype(np.float32)
    return out


def random_blob(codes_dim: int = 6, seed: int = 0) -> np.ndarray:
    return pack(random_params(codes_dim, seed), codes_dim)


def params_keys_conversion(dict_params: Dict, key_name: str = "forward_vq3_d/") -> Dict:
    """Mirror of `scripts/inference_runner.py:153-165`: strip the training-wrapper prefix."""
    for key in list(dict_params.keys()):
        if key_name in key:
            dict_params[key.split(key_name)[1]] = dict_params.pop(key)
    return dict_params


def load_params_npz(filename: str, names: List[Tuple[str, str]]) -> Dict[str, Dict[str, np.ndarray]]:
    """`params.npz` (leaves `arr_0..`, JAX dict-flatten order = sorted keys) → nested dict.

    `names` is the full ordered (module, param) list of the checkpoint's tree (the pickled
    jaxlib PyTreeDef in `state_variables.npy` is not unpickled here). Mirror of
    `scripts/inference_runner.py:136-150` without `jax.tree_util.tree_unflatten`.
    """
    with np.load(filename, allow_pickle=False) as f:
        files = sorted(f.files, key=lambda s: int(s.split("_")[1]) if s.startswith("arr_") else s)
        if len(files) != len(names):
            raise ValueError(f"{filename}: {len(files)} arrays but {len(names)} names")
        out: Dict[str, Dict[str, np.ndarray]] = {}
        for (mod, name), fn in zip(names, files):
            out.setdefault(mod, {})[name] = np.asarray(f[fn])
    return params_keys_conversion(out)


def save_params_npz(filename: str, params: Dict[str, Dict[str, np.ndarray]]) -> List[Tuple[str, str]]:
    """Write params in the reference's npz leaf order (sorted module, then sorted param)."""
    names = [(m, p) for m in sorted(params) for p in sorted(params[m])]
    np.savez(filename, *[params[m][p] for m, p in names])
    return names
