"""The drop-in boundary of the reference's script entry points, on CPU:
`scripts/tokenize_pdb.py:main` / `scripts/decode_tokens.py:main` signatures and the model
selection from `config_overrides` (`/root/reference/scripts/tokenize_pdb.py:32-45, 109-119`).
The per-device compute is the CPU oracle stand-in of test_host.py; the CLI and runner code are
the product's."""
import inspect
import os
import sys

import numpy as np
import pytest

from pst_amd import config as C
from pst_amd import params as P
from pst_amd import runner, synthetic

from test_host import OracleTokenizeFn, _oracle_tokens, _write

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd", "scripts"))
import decode_tokens  # noqa: E402
import tokenize_pdb  # noqa: E402


@pytest.mark.parametrize("cb,df", sorted(C.SHIPPED))
def test_overrides_select_every_shipped_model(cb, df):
    assert C.config_from_overrides(C.overrides_for(cb, df)) == C.tokenizer_config(cb, df)
    # the model override alone carries df; ".yaml" may be omitted as in Hydra
    assert C.config_from_overrides([f"model=gnn/ablation_{C.CODEBOOK_SURNAME[cb]}_df_{df}"]) == \
        C.tokenizer_config(cb, df)


def test_overrides_defaults_and_inert_keys():
    assert C.config_from_overrides(None) == C.tokenizer_config(4096, 1)
    assert C.config_from_overrides([]) == C.tokenizer_config(4096, 1)
    assert C.config_from_overrides(["data=ablation_df_1.yaml"]) == C.tokenizer_config(4096, 1)
    got = C.config_from_overrides(C.overrides_for(64000, 4) + ["random_seed=7", "mixed_precision=false",
                                                               "model.weight_paths=/w/64k"])
    assert (got.codebook_size, got.downsampling_ratio, got.weight_dir) == (64000, 4, "/w/64k")


@pytest.mark.parametrize("bad", [
    ["model=gnn/ablation_8k_df_1.yaml"],                                  # no such model
    ["model=ablation_4k_df_1.yaml"],                                      # the reference's broken default path
    ["model=gnn/ablation_0.5k_df_2.yaml", "data=ablation_df_2.yaml"],     # not shipped
    ["model=gnn/ablation_64k_df_4.yaml", "data=ablation_df_2.yaml"],      # df disagree
    ["data=ablation_df_4.yaml"],                                          # df 4 data on the df 1 default model
    ["data=ablation_1.yaml"],
    ["optimizer=adam"],
    ["data.downsampling_ratio=2"],
    ["model"],
])
def test_overrides_unrecognised_raise(bad):
    with pytest.raises(ValueError):
        C.config_from_overrides(bad)


def test_overrides_continuous_model_not_tokenizable():
    with pytest.raises(NotImplementedError):
        C.config_from_overrides(["model=gnn/ablation_continuous_df_1.yaml", "data=ablation_df_1.yaml"])


@pytest.mark.reference
@pytest.mark.parametrize("cb,df", sorted(C.SHIPPED))
def test_overrides_equal_hydra_composition(cb, df):
    """Without the YAML tree, the same model as composing the reference's tree with Hydra's rules."""
    import _refenv
    ref = C.config_from_hydra(C.load_config("vq3d_inference", overrides=C.overrides_for(cb, df),
                                            config_path=os.path.join(_refenv.REF, "config", "structure_tokenizer")))
    assert C.config_from_overrides(C.overrides_for(cb, df)) == ref


def test_main_signatures_match_reference():
    """Positional parameters as the reference's (tokenize_pdb.py:32-39, decode_tokens.py:32-38);
    the extras are keyword-only."""
    def pos(f):
        return [p.name for p in inspect.signature(f).parameters.values()
                if p.kind == p.POSITIONAL_OR_KEYWORD]

    def kwonly(f):
        return {p.name for p in inspect.signature(f).parameters.values() if p.kind == p.KEYWORD_ONLY}

    assert pos(tokenize_pdb.main) == ["pdbs", "token_save_path", "backend", "batch_size_per_device",
                                      "config_name", "config_overrides"]
    assert inspect.signature(tokenize_pdb.main).parameters["batch_size_per_device"].default == 8
    assert kwonly(tokenize_pdb.main) == {"weights_dir", "config_path"}
    assert pos(decode_tokens.main) == ["sequences", "structure_save_path", "backend", "batch_size_per_device",
                                       "config_overrides"]
    assert kwonly(decode_tokens.main) == {"weights_dir", "config_path"}


@pytest.fixture
def oracle_runner(monkeypatch):
    seen = {}

    def prep(cfg, devices, emit_aux=False):
        seen["cfg"] = cfg
        return OracleTokenizeFn(cfg, devices)
    monkeypatch.setattr(runner.InferenceRunner, "prepare_devices", staticmethod(lambda backend="gpu": ([0], 1)))
    monkeypatch.setattr(runner.InferenceRunner, "prepare_tokenize_fn", staticmethod(prep))
    return seen


def test_main_reference_call_selects_model_from_overrides(tmp_path, oracle_runner):
    """A reference-style call (positional config_name, overrides naming 64k / df 4) tokenizes
    with codebook 64 000, df 4 — no config_path needed."""
    cfg = C.tokenizer_config(64000, 4)
    D = len(cfg.levels)
    mdir = tmp_path / "model"
    mdir.mkdir()
    P.save_params_npz(str(mdir / "params.npz"), P.random_full_params(D, seed=3))
    ss = [synthetic.synthetic_protein(n, 90 + n) for n in (57, 66, 83)]
    pdbs = [_write(tmp_path, f"p{i}.pdb", s) for i, s in enumerate(ss)]
    out = str(tmp_path / "tok")
    tokenize_pdb.main(pdbs, out, "gpu", 2, None,
                      ["model=gnn/ablation_64k_df_4.yaml", "data=ablation_df_4.yaml"], weights_dir=str(mdir))
    assert oracle_runner["cfg"] == cfg
    blob = P.pack(P.params_keys_conversion(P.random_full_params(D, seed=3)), D)
    for i, s in enumerate(ss):
        t = np.load(os.path.join(out, f"p{i}_tokens.npy"))
        assert t.shape == (1, s.nb_residues // 4)
        assert np.array_equal(t[0], _oracle_tokens(blob, cfg, s))


def test_main_unknown_override_raises_before_any_work(tmp_path, oracle_runner):
    out = tmp_path / "tok"
    with pytest.raises(ValueError):
        tokenize_pdb.main([], str(out), "gpu", config_overrides=["model=gnn/ablation_2k_df_1.yaml"])
    assert not out.exists() and "cfg" not in oracle_runner


AE_GOLD = os.path.join(ROOT, "tests", "golden", "ae_ref.npz")


@pytest.mark.skipif(not os.path.exists(AE_GOLD), reason="ae_ref.npz not generated")
def test_ae_fixture_tokens_equal_oracle_and_layout():
    """The reference's autoencoder pass (`make_ae_golden.py`): its tokens equal the C oracle's on
    the same inputs and weights, the node count is not a multiple of df where the case says so,
    the atom mask is the backbone of the kept residues, and the UNK residue's atoms are zero."""
    from oracle import oracle as O
    F = np.load(AE_GOLD)
    for c in sorted({k.split("/")[0] for k in F.files}):
        n, n_node, T, cb, df, D, pseed = (int(v) for v in F[c + "/meta"])
        pos = F[c + "/in_positions"].astype(np.float64)
        fl = F[c + "/in_flags"]
        blob = P.pack(P.params_keys_conversion(P.random_full_params(D, pseed)), D)
        got = O.tokenize(blob, C.LEVELS[cb], df, pos, fl)
        assert got["graph"]["n"] == n_node and len(got["tokens"]) == T
        assert np.array_equal(got["tokens"], F[c + "/tokens"]), c
        mask = F[c + "/final_atom_mask"]
        assert mask.shape == (512, 37) and mask[:n_node][:, [0, 1, 2, 4]].all() and mask.sum() == 4 * n_node
        aa = F[c + "/in_aatype"]
        kept = np.all(fl[:, [0, 1, 2, 4]] & 1, axis=1)
        unk = np.nonzero(aa[kept] == 20)[0]
        atoms = F[c + "/final_atom_positions"]
        assert len(unk) == 1 and np.all(atoms[unk] == 0) and np.all(atoms[:, [3] + list(range(5, 37))] == 0)
        if df > 1:
            assert n_node % df != 0
