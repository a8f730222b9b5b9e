"""Decode-path fixtures from the reference itself (float64 under the NumPy shim).

For each case, token ids → `Vq3D.indexes_to_codes` → `Vq3D.decode` → `structure_module`
(the two halves of `decode_and_make_structure`, model/model.py:481-569, called separately to
keep the intermediates) with `random_full_params` weights, at the reference's own padding
(512 node slots). Stores the real rows of: codes, up-projected codes, upsampled single
representation (s_i), pair representation z_ij, the 8 per-layer affines (traj), backbone
torsion sin/cos, atom14 positions and final atom37 positions. ~10 minutes per case.

    python tests/golden/make_decode_golden.py          # decode_golden_f64.npz (2 small cases)
    python tests/golden/make_decode_golden.py wide     # decode_ref_wide.npz (128-512 tokens)

The wide cases keep the pair representation only for PAIR_ROWS rows i (all j) to stay small.
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

# (name, codebook, df, n_tokens, token seed, param seed)
CASES = [("dec_k4096_df1_t40", 4096, 1, 40, 1, 77), ("dec_k64000_df4_t14", 64000, 4, 14, 2, 78)]
# 128-512 tokens, df 1 / 2 / 4, two level sets (decode depth)
CASES_WIDE = [("dec_k4096_df1_t128", 4096, 1, 128, 11, 81), ("dec_k4096_df1_t512", 4096, 1, 512, 12, 82),
              ("dec_k64000_df4_t128", 64000, 4, 128, 13, 83), ("dec_k4096_df2_t256", 4096, 2, 256, 14, 84)]
PAIR_ROWS = 4


def main(wide=False):
    import _refenv
    _refenv.activate(f64=True)
    import numpy as np
    import haiku as hk
    from structure_tokenizer.model.model import Vq3D
    from pst_amd import params as P
    from pst_amd.config import LEVELS, load_config, overrides_for

    out = {}
    wide_path = os.path.join(HERE, "decode_ref_wide.npz")
    if wide and os.path.exists(wide_path):  # resume: keep the cases already made
        with np.load(wide_path) as old:
            out = {k: old[k] for k in old.files}
    for name, cb, df, T, tseed, pseed in (CASES_WIDE if wide else CASES):
        if name + "/meta" in out:
            continue
        t0 = time.time()
        cfg = load_config("vq3d_inference", overrides=overrides_for(cb, df),
                          config_path=os.path.join(_refenv.REF, "config", "structure_tokenizer"))
        D = len(LEVELS[cb])
        params = {k: {n: np.asarray(v, np.float64) for n, v in d.items()} for k, d in P.random_full_params(D, pseed).items()}
        rng = np.random.default_rng(tseed)
        Tpad = 512 // df
        tokens = np.full((1, Tpad), 4097, np.int64)
        tokens[0, :T] = rng.integers(0, cb, T)
        tokens_mask = np.zeros((1, Tpad, 1))
        tokens_mask[0, :T] = 1
        nodes_mask = np.zeros((1, 512, 1))
        nodes_mask[0, :T * df] = 1

        def fn(tok, nm, tm):
            m = Vq3D(config=cfg.model, global_config=cfg.data)
            codes = m.indexes_to_codes(tok)
            qp, s_i, z = m.decode(codes, nm, tm, is_training=False, safe_key=None)
            b, n = s_i.shape[0], s_i.shape[1]
            gt = np.concatenate([np.ones((b, n, 3)), np.zeros((b, n, 1)), np.ones((b, n, 1)), np.zeros((b, n, 32))], -1)
            aat = np.concatenate([np.ones((b, n, 1)), np.zeros((b, n, 20))], -1)
            st = m.structure_module({"single": s_i, "pair": z}, {"atom37_gt_exists": gt, "aatype": aat}, nm)
            return codes, qp, s_i, z, st

        codes, qp, s_i, z, st = hk.transform(fn).apply(params, None, tokens, nodes_mask, tokens_mask)
        N = T * df
        pre = name + "/"
        out[pre + "meta"] = np.array([cb, df, T, N, D, pseed], np.int64)
        out[pre + "tokens"] = tokens[0, :T].astype(np.uint32)
        out[pre + "codes"] = np.asarray(codes)[0, :T].astype(np.float32)
        out[pre + "up_proj"] = np.asarray(qp)[0, :T].astype(np.float32)
        out[pre + "single"] = np.asarray(s_i)[0, :N].astype(np.float32)
        if wide:  # rows 0, N/3, 2N/3, N-1 of z_ij (all j)
            rows = np.unique(np.linspace(0, N - 1, PAIR_ROWS).astype(np.int64))
            out[pre + "pair_rows"] = rows
            out[pre + "pair"] = np.asarray(z)[0, rows, :N].astype(np.float32)
        else:
            out[pre + "pair"] = np.asarray(z)[0, :N, :N].astype(np.float32)
        out[pre + "traj"] = np.asarray(st["traj"])[0, :, :N].astype(np.float32)
        out[pre + "angles"] = np.asarray(st["sidechains"]["angles_sin_cos"])[0, :, :N].astype(np.float32)
        ap = st["sidechains"]["atom_pos"]
        out[pre + "atom14"] = np.stack([np.asarray(ap.x), np.asarray(ap.y), np.asarray(ap.z)], -1)[0, -1, :N].astype(np.float32)
        out[pre + "atom37"] = np.asarray(st["final_atom_positions"])[0, :N].astype(np.float32)
        out[pre + "atom37_mask"] = np.asarray(st["final_atom_mask"])[0, :N].astype(np.uint8)
        print(name, "done in", round(time.time() - t0), "s", flush=True)
        if wide:  # checkpoint after every case (each takes minutes)
            np.savez_compressed(wide_path, **out)
    if not wide:
        np.savez_compressed(os.path.join(HERE, "decode_golden_f64.npz"), **out)


if __name__ == "__main__":
    main(wide=len(sys.argv) > 1 and sys.argv[1] == "wide")
