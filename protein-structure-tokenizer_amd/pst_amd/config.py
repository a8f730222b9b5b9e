"""Configuration for the tokenize path.

Two entry points:
  * `load_config(name, job_name, overrides, config_path)` — mirror of
    `structure_tokenizer/utils/utils.py:47-58` (Hydra compose) for users who keep the
    reference's YAML tree: PyYAML + the `defaults:` list merge Hydra applies (defaults first,
    then the file's own keys; `group=file.yaml` overrides replace a group's default).
  * `tokenizer_config(codebook_size, df)` — the hot-path hyper-parameters of the shipped
    models (`config/structure_tokenizer/model/gnn/ablation_*_df_*.yaml` over
    `model/shared.yaml`, `data/ablation_df_*.yaml`) as a plain dataclass, so the runtime does not
    need the YAML tree.
"""
import copy
import dataclasses
import os
from typing import Dict, List, Optional, Sequence, Tuple

import yaml

CODEBOOK_SURNAME = {432: "0.5k", 1728: "1.7k", 4096: "4k", 64000: "64k"}
LEVELS = {
    432: (4, 4, 3, 3, 3),
    1728: (4, 4, 4, 3, 3, 3),
    4096: (4, 4, 4, 4, 4, 4),
    64000: (8, 8, 8, 5, 5, 5),
}
# (codebook, df) pairs with a shipped model config (tokenize_pdb.py:102-113 picks by name)
SHIPPED = {(432, 1), (1728, 1), (4096, 1), (4096, 2), (4096, 4), (64000, 1), (64000, 2), (64000, 4)}


@dataclasses.dataclass(frozen=True)
class TokenizerConfig:
    codebook_size: int = 4096
    downsampling_ratio: int = 1
    levels: Tuple[int, ...] = LEVELS[4096]
    seq_max_size: int = 512          # data.seq_max_size
    graph_max_neighbor: int = 50     # data.graph_max_neighbor
    residue_loc_is_alphac: bool = True
    pad_token_id: int = 4097
    hidden: int = 128                # encoder.encoding_dimension == gnn hidden_dimension
    pe_dim: int = 128                # encoder.positional_encoding_dimension
    gnn_layers: int = 3
    num_head: int = 4                # down_sampler.cross_attn.num_head
    sc_num_block: int = 3            # down_sampler.sc_num_block
    transition_factor: int = 2       # *_transition.num_intermediate_factor
    use_local_attn: bool = True
    weight_dir: str = "weights/4k_df_1/"

    @property
    def codes_dimension(self) -> int:
        return len(self.levels)

    @property
    def max_out_len(self) -> int:
        return self.seq_max_size // self.downsampling_ratio


def config_from_hydra(cfg) -> TokenizerConfig:
    """The composed `vq3d_inference` config (`load_config`, as `scripts/tokenize_pdb.py:41-46`
    builds it) → TokenizerConfig. Reads cfg.model.model.codebook.levels,
    cfg.model.weight_paths and cfg.data.data.*; rejects settings the device path does not
    implement (continuous / non-FSQ models)."""
    m = cfg["model"]
    d = cfg["data"]["data"]
    cb = m["model"]["codebook"]
    if not cb.get("use_codebook", True) or cb.get("method", "fsq") != "fsq":
        raise NotImplementedError("only FSQ codebook models are tokenized by libpst")
    levels = tuple(int(x) for x in cb["levels"])
    return TokenizerConfig(
        codebook_size=int(cb.get("num_codes", 0)) or int(__import__("math").prod(levels)),
        downsampling_ratio=int(d["downsampling_ratio"]), levels=levels,
        seq_max_size=int(d["seq_max_size"]), graph_max_neighbor=int(d["graph_max_neighbor"]),
        residue_loc_is_alphac=bool(d["graph_residue_loc_is_alphac"]),
        pad_token_id=int(d.get("pad_token_id", 4097)), weight_dir=str(m.get("weight_paths", "")))


def tokenizer_config(codebook_size: int = 4096, df: int = 1) -> TokenizerConfig:
    if (codebook_size, df) not in SHIPPED:
        raise ValueError(f"no shipped model for codebook_size={codebook_size}, df={df}")
    return TokenizerConfig(
        codebook_size=codebook_size, downsampling_ratio=df, levels=LEVELS[codebook_size],
        weight_dir=f"weights/{CODEBOOK_SURNAME[codebook_size]}_df_{df}/")


# ---------------------------------------------------------------- YAML loader (Hydra subset)
class ConfigDict(dict):
    """Attribute-access dict (what the reference reads through `ml_collections.ConfigDict`)."""

    def __init__(self, d=None):
        super().__init__()
        for k, v in (d or {}).items():
            self[k] = ConfigDict(v) if isinstance(v, dict) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


def _deep_merge(base: Dict, over: Dict) -> Dict:
    out = copy.deepcopy(base)
    for k, v in over.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _deep_merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def _load_yaml(path: str) -> Dict:
    with open(path) as fh:
        return yaml.safe_load(fh) or {}


def _compose(root: str, group: Optional[str], name: str, choices: Dict[str, str]) -> Dict:
    rel = name if name.endswith(".yaml") else name + ".yaml"
    path = os.path.join(root, group, rel) if group else os.path.join(root, rel)
    node = _load_yaml(path)
    defaults = node.pop("defaults", []) or []
    merged: Dict = {}
    for d in defaults:
        if isinstance(d, dict):
            (g, default_name), = d.items()
            sel = choices.get(g, default_name)
            merged = _deep_merge(merged, {g: _compose(root, g, sel, choices)})
        else:  # same-group default, e.g. `- shared` inside model/gnn/x.yaml
            merged = _deep_merge(merged, _compose(root, group, d, choices))
    return _deep_merge(merged, node)


def load_config(name: str, job_name: str = "tokenize", overrides: Optional[Sequence[str]] = None,
                config_path: str = "config/structure_tokenizer") -> ConfigDict:
    choices = {}
    for o in overrides or []:
        k, v = o.split("=", 1)
        choices[k] = v
    return ConfigDict(_compose(config_path, None, name, choices))


def overrides_for(codebook_size: int, df: int) -> List[str]:
    """The overrides `scripts/tokenize_pdb.py:109-113` builds."""
    return [f"model=gnn/ablation_{CODEBOOK_SURNAME[codebook_size]}_df_{df}.yaml",
            f"data=ablation_df_{df}.yaml"]


_SURNAME_TO_CODEBOOK = {v: k for k, v in CODEBOOK_SURNAME.items()}
# top-level keys of vq3d_inference.yaml that a Hydra override may set and that do not reach the
# tokenize computation (the inference path draws no random numbers; mixed precision is off in
# every shipped config and libpst computes in f32 regardless)
_INERT_KEYS = {"random_seed", "mixed_precision", "deterministic", "use_remat", "zero_init"}


def _override_file(group: str, value: str, pattern: str) -> Tuple[str, int]:
    import re
    m = re.fullmatch(pattern, value[:-5] if value.endswith(".yaml") else value)
    if not m:
        raise ValueError(f"unrecognised {group} override {group}={value!r}: the shipped configs are "
                         + ("gnn/ablation_{0.5k,1.7k,4k,64k}_df_{1,2,4}.yaml" if group == "model"
                            else "ablation_df_{1,2,4}.yaml"))
    return m.group(1) if m.lastindex and m.lastindex > 1 else "", int(m.group(m.lastindex))


def config_from_overrides(config_overrides: Optional[Sequence[str]] = None,
                          weight_dir: Optional[str] = None) -> TokenizerConfig:
    """The model the reference's `main(..., config_overrides=...)` composes
    (`scripts/tokenize_pdb.py:40-45, 109-113`), without the YAML tree: (codebook, df) come from
    `model=gnn/ablation_<K>_df_<df>.yaml` and `data=ablation_df_<df>.yaml`.

    * `None` / `[]`: codebook 4096, df 1. (The reference's own defaults list names
      `model: ablation_4k_df_1.yaml` / `data: ablation_1.yaml`, files that do not exist at those
      paths, so its bare call fails in Hydra; 4k / df 1 is what those names intend.)
    * only `model=…`: df from the model's name (its `max_out_len` = 512 / df).
    * model and data naming different df: ValueError (the model's query PE table and the data's
      token count disagree).
    * `model.weight_paths=DIR` sets the weights directory; the inert top-level keys
      (`random_seed`, `mixed_precision`, `deterministic`, `use_remat`, `zero_init`) are accepted.
    * anything else (other groups, `ablation_continuous_*` models, malformed entries): ValueError
      or, for continuous models, NotImplementedError — never a silent default.
    """
    cb: Optional[int] = None
    df_model: Optional[int] = None
    df_data: Optional[int] = None
    for o in config_overrides or []:
        if not isinstance(o, str) or "=" not in o:
            raise ValueError(f"malformed config override {o!r} (expected key=value)")
        k, v = o.split("=", 1)
        k = k.strip().lstrip("+")
        v = v.strip()
        if k == "model":
            if "continuous" in v:
                raise NotImplementedError(f"{o}: continuous (codebook-free) models emit no tokens")
            name, df_model = _override_file("model", v, r"gnn/ablation_(0\.5k|1\.7k|4k|64k)_df_(\d+)")
            cb = _SURNAME_TO_CODEBOOK[name]
        elif k == "data":
            _, df_data = _override_file("data", v, r"ablation_df_(\d+)")
        elif k == "model.weight_paths":
            weight_dir = v
        elif k in _INERT_KEYS:
            continue
        else:
            raise ValueError(f"unrecognised config override {o!r}")
    if df_model is not None and df_data is not None and df_model != df_data:
        raise ValueError(f"model override is df {df_model} but data override is df {df_data}")
    if cb is None and df_data not in (None, 1):
        raise ValueError(f"data=ablation_df_{df_data}.yaml needs a matching model= override "
                         "(the default model is ablation_4k_df_1)")
    df = df_model if df_model is not None else (df_data or 1)
    cfg = tokenizer_config(4096 if cb is None else cb, df)
    if weight_dir:
        cfg = dataclasses.replace(cfg, weight_dir=weight_dir)
    return cfg
