"""Encoder-half parameters: haiku names, shapes, the flat blob the C ABI takes, random init.

Names are the haiku paths the reference creates for `Vq3D.encode_and_quantize` after
`params_keys_conversion` strips `forward_vq3_d/` (`scripts/inference_runner.py:153-165`);
`tests/test_params.py` checks them (and the decoder half) against the reference model
initialised under the test shim (`tests/golden/full_param_names.json`). The blob is every tensor below, row-major, concatenated in `param_spec` order — the
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
    s += _scaler_spec(DS, n_block)
    s += [("vq3_d/down_proj", "w", (H, codes_dim)), ("vq3_d/down_proj", "b", (codes_dim,))]
    return s


US = "vq3_d/~/cross_attn_upsampling"
SEQ = "vq3_d/~/sequence_decoder"
SM = "vq3_d/~/structure_module"


def _scaler_spec(root: str, B: int) -> List[Tuple[str, str, Tuple[int, ...]]]:
    s: List[Tuple[str, str, Tuple[int, ...]]] = []
    for nm in ("query_norm", "data_norm"):
        s += [(f"{root}/cross_attention/{nm}", "scale", (B, H)), (f"{root}/cross_attention/{nm}", "offset", (B, H))]
    att = f"{root}/cross_attention/attention"
    for w in ("query_w", "key_w", "value_w", "gating_w"):
        s += [(att, w, (B, H, 4, 32))]
    s += [(att, "gating_b", (B, 4, 32)), (att, "output_w", (B, 4, 32, H)), (att, "output_b", (B, H))]
    for tr in ("resampled_transition", "original_transition"):
        s += [(f"{root}/{tr}/input_layer_norm", "scale", (B, H)), (f"{root}/{tr}/input_layer_norm", "offset", (B, H))]
        s += [(f"{root}/{tr}/transition1", "weights", (B, H, 2 * H)), (f"{root}/{tr}/transition1", "bias", (B, 2 * H))]
        s += [(f"{root}/{tr}/transition2", "weights", (B, 2 * H, H)), (f"{root}/{tr}/transition2", "bias", (B, H))]
    return s


def _lin(mod: str, fi: int, fo: int, w: str = "weights", b: str = "bias"):
    return [(mod, w, (fi, fo)), (mod, b, (fo,))]


def _ln(mod: str, n: int = H):
    return [(mod, "scale", (n,)), (mod, "offset", (n,))]


def decoder_param_spec(codes_dim: int = 6, n_block: int = 3) -> List[Tuple[str, str, Tuple[int, ...]]]:
    """Decoder-half tensors (`Vq3D.decode_and_make_structure`, model/model.py:481-570).

    Not used by the tokenize path; listed so a full `params.npz` (189 leaves) can be split by
    leaf order. Names/shapes: tests/golden/full_param_names.json (reference model initialised
    under the test shim, see tests/golden/make_param_names.py).
    """
    S = 384
    s = _lin("vq3_d/up_proj", codes_dim, H, "w", "b")
    s += _scaler_spec(f"{US}/cross_attn_scaler_iteration", n_block)
    s += _lin(f"{US}/linear_proj_original", 2 * H, H, "w", "b")
    s += _lin(f"{SEQ}/linear", 2 * H, H, "w", "b")
    s += _ln(f"{SEQ}/pair_transition_init/input_layer_norm")
    s += _lin(f"{SEQ}/pair_transition_init/transition1", H, 2 * H)
    s += _lin(f"{SEQ}/pair_transition_init/transition2", 2 * H, H)
    pr = f"{SEQ}/pairwise_representation"
    s += _ln(f"{pr}/layer_norm_input") + _ln(f"{pr}/layer_norm_output")
    s += _lin(f"{pr}/left_projection", H, 2 * H) + _lin(f"{pr}/right_projection", H, 2 * H)
    s += _lin(f"{pr}/right_projection_1", 2 * H, H)
    s += _lin(f"{pr}/output_projection_layer1", 2 * H, 2 * H) + _lin(f"{pr}/output_projection_layer2", 2 * H, H)
    fi = f"{SM}/fold_iteration"
    s += _lin(f"{fi}/affine_update", S, 6) + _ln(f"{fi}/attention_layer_norm", S)
    ipa = f"{fi}/invariant_point_attention"
    s += [(ipa, "trainable_point_weights", (12,))]
    s += _lin(f"{ipa}/attention_2d", H, 12) + _lin(f"{ipa}/kv_point_local", S, 432)
    s += _lin(f"{ipa}/kv_scalar", S, S) + _lin(f"{ipa}/output_projection", 2112, S)
    s += _lin(f"{ipa}/q_point_local", S, 144) + _lin(f"{ipa}/q_scalar", S, 192)
    rs = f"{fi}/rigid_sidechain"
    s += _lin(f"{rs}/input_projection", S, H) + _lin(f"{rs}/input_projection_1", H, H)
    for r in ("resblock1", "resblock1_1", "resblock2", "resblock2_1"):
        s += _lin(f"{rs}/{r}", H, H)
    s += _lin(f"{rs}/unnormalized_angles", H, 6)
    for t in ("transition", "transition_1", "transition_2"):
        s += _lin(f"{fi}/{t}", S, S)
    s += _ln(f"{fi}/transition_layer_norm", S)
    s += _lin(f"{SM}/initial_projection", H, S) + _ln(f"{SM}/pair_layer_norm") + _ln(f"{SM}/single_layer_norm")
    return s


def full_param_spec(codes_dim: int = 6) -> List[Tuple[str, str, Tuple[int, ...]]]:
    """Every leaf of a Vq3D checkpoint in JAX dict-flatten order (sorted module, sorted name).

    This is the leaf order of `params.npz` (`scripts/inference_runner.py:146-149` unflattens
    `uploaded.files` in order against the checkpoint's treedef; `ForwardVQ3D` wraps exactly one
    `Vq3D`, model/model.py:575-624, so its `forward_vq3_d/` prefix does not change the order).
    """
    s = param_spec(codes_dim) + decoder_param_spec(codes_dim)
    return sorted(s, key=lambda t: (t[0], t[1]))


def decoder_param_count(codes_dim: int = 6) -> int:
    return int(sum(np.prod(sh) for _, _, sh in decoder_param_spec(codes_dim)))


def pack_decoder(params: Dict[str, Dict[str, np.ndarray]], codes_dim: int = 6) -> np.ndarray:
    """Decoder-half tensors → contiguous float32 blob in `decoder_param_spec` order
    (the layout `pst_decoder_create` takes)."""
    parts = []
    for mod, name, shape in decoder_param_spec(codes_dim):
        try:
            a = np.asarray(params[mod][name], dtype=np.float32)
        except KeyError as e:
            raise KeyError(f"missing parameter {mod}/{name}") from e
        if a.shape != shape:
            raise ValueError(f"{mod}/{name}: expected shape {shape}, got {a.shape}")
        parts.append(a.reshape(-1))
    return np.ascontiguousarray(np.concatenate(parts))


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


def random_full_params(codes_dim: int = 6, seed: int = 0) -> Dict[str, Dict[str, np.ndarray]]:
    """A whole Vq3D checkpoint's worth of random tensors (stands in for a real `params.npz`,
    which is not available offline). Encoder as `random_params`; decoder weights truncated
    normal with σ = 1/sqrt(fan_in), biases / LN offsets N(0, 0.1²), LN scales 1 + N(0, 0.1²),
    IPA point weights softplus⁻¹(1) + N(0, 0.1²) — activations stay O(1) through the decoder
    and structure module, so decode parity tests exercise every path."""
    out = random_params(codes_dim, seed)
    rng = np.random.default_rng(seed + 1)
    for mod, name, shape in decoder_param_spec(codes_dim):
        stacked = mod.startswith(US + "/cross_attn_scaler_iteration")
        core = shape[1:] if stacked else shape
        if name in ("w", "weights", "query_w", "key_w", "value_w", "gating_w", "output_w"):
            fan_in = core[0] * core[1] if name == "output_w" else core[0]
            v = np.clip(rng.standard_normal(shape), -2, 2) / np.sqrt(fan_in)
        elif name == "scale":
            v = 1.0 + 0.1 * rng.standard_normal(shape)
        elif name in ("gating_b",):
            v = 1.0 + 0.1 * rng.standard_normal(shape)
        elif name == "trainable_point_weights":
            v = np.log(np.e - 1.0) + 0.1 * rng.standard_normal(shape)
        else:
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


def load_params_npz(filename: str, names=None, codes_dim=None, convert: bool = True
                    ) -> Dict[str, Dict[str, np.ndarray]]:
    """`params.npz` → nested haiku-style dict. Mirror of `scripts/inference_runner.py:136-150`.

    The reference unflattens the arrays, in `uploaded.files` order, against the PyTreeDef
    pickled in `state_variables.npy`. That pickle is never loaded here (only loaders that
    execute nothing from the file are used); the tree is instead `names` (ordered
    (module, param) pairs), by default `full_param_spec(codes_dim)` — the leaf order JAX
    gives a Vq3D params dict; `codes_dim` defaults to the length of the first leaf
    (`vq3_d/down_proj/b`). An npz keyed `module:param` (`save_params_npz(..., named=True)`)
    is read by name. Every array's shape is checked against the spec; `convert` applies
    `params_keys_conversion` as `InferenceRunner.load_params` does.
    """
    with np.load(filename, allow_pickle=False) as f:
        files = list(f.files)
        out: Dict[str, Dict[str, np.ndarray]] = {}
        if files and all(":" in k for k in files):
            for k in files:
                mod, name = k.rsplit(":", 1)
                out.setdefault(mod, {})[name] = np.asarray(f[k])
        else:
            if names is None:
                if codes_dim is None:
                    codes_dim = int(f[files[0]].shape[0]) if files and f[files[0]].ndim == 1 else 6
                names = [(m, p) for m, p, _ in full_param_spec(codes_dim)]
            if len(files) != len(names):
                raise ValueError(f"{filename}: {len(files)} arrays but the tree has {len(names)} leaves")
            for (mod, name), fn in zip(names, files):
                out.setdefault(mod, {})[name] = np.asarray(f[fn])
    conv = params_keys_conversion(dict(out))
    if codes_dim is None:
        b = conv.get("vq3_d/down_proj", {}).get("b")
        codes_dim = int(b.shape[0]) if b is not None else 6
    spec = {(m, p): sh for m, p, sh in full_param_spec(codes_dim)}
    for mod, d in conv.items():
        for name, a in d.items():
            want = spec.get((mod, name))
            if want is not None and tuple(a.shape) != tuple(want):
                raise ValueError(f"{filename}: {mod}/{name} has shape {a.shape}, expected {want}")
    return conv if convert else out


def save_params_npz(filename: str, params: Dict[str, Dict[str, np.ndarray]], named: bool = False) -> List[Tuple[str, str]]:
    """Write params in the reference's npz leaf order (sorted module, then sorted param):
    `arr_0..` like a flattened JAX tree, or keyed `module:param` when `named`."""
    names = [(m, p) for m in sorted(params) for p in sorted(params[m])]
    if named:
        np.savez(filename, **{f"{m}:{p}": params[m][p] for m, p in names})
    else:
        np.savez(filename, *[params[m][p] for m, p in names])
    return names
