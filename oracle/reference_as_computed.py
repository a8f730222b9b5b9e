"""The reference's tokenize forward AS THE REFERENCE COMPUTES IT, in PyTorch-CPU float32.

TEST INFRASTRUCTURE / CPU BASELINE ONLY: imported by tests/ and by bench.py's
cpu_baseline leg; the product never loads it.

Where `oracle/pst_oracle.c` restates the path in the GPU's canonical operation order on the
real residues only, this module follows the reference's own shapes and work:
`preprocess_sample` pads every protein to 512 nodes and 25 600 edge slots
(`preprocessing.py:191-283`), the edge positional encoding is evaluated per edge
(`positional_encoding_layer.py:49-150`), the three MPNN layers run over all padded edges
(`gnn_layers.py:325-438`, MaskedLayerNorm `:79-164`), the downsampler's cross-attention is dense
over the 512 keys with the local mask as an additive −1e9 bias (`model.py:264-318, 357-420`,
`modules.py:199-636`), and the FSQ codebook materialises `distances` / `soft_proba` over all K
codes and the perplexity histogram (`quantize.py:141-244`). Matmuls are plain float32 torch
(oneDNN/MKL reductions); the graph itself comes from the C oracle (it equals the reference's
bitwise, tests/test_oracle_golden.py) and is padded by `pst_amd.graph.pad_protein_graph`.

Used (1) as the "reference-as-computed" CPU baseline timed by bench.py and (2) as an independent
float32 implementation whose token ids are checked against the reference fixtures.
"""
import math
from typing import Dict, Sequence

import numpy as np
import torch

P_NODES, K_NB, H = 512, 50, 128


def _pe(x: torch.Tensor, n: int) -> torch.Tensor:
    """Sinusoidal PE of integer positions x [...] → [..., 128], float32 argument as under JAX."""
    k = torch.arange(1, H + 1)
    num = torch.where(k % 2 == 1, 2 * (k - 1), 2 * k).to(torch.float32)
    pw = torch.pow(torch.tensor(float(n), dtype=torch.float64), (num / H).to(torch.float64)).to(torch.float32)
    arg = (x.to(torch.float32)[..., None] * torch.tensor(math.pi, dtype=torch.float32)) / pw
    return torch.where(k % 2 == 1, torch.cos(arg), torch.sin(arg))


def _gelu(x):
    return torch.nn.functional.gelu(x, approximate="tanh")


def _ln(x, s, o, eps=1e-5):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return s * torch.rsqrt(var + eps) * (x - mu) + o


def _masked_ln(x, mask, s, o, eps=1e-5):
    x = mask * x
    mu = (mask * x).mean(-1, keepdim=True)
    var = (mask * ((x - mu) * (x - mu))).mean(-1, keepdim=True)
    return s * torch.rsqrt(var + eps) * (x - mu) + o


class ReferenceAsComputed:
    """Vq3D.encode_and_quantize for one (codebook levels, df) on CPU, weights from a params dict
    shaped like `pst_amd.params.random_params` (haiku module/leaf names)."""

    def __init__(self, params: Dict[str, Dict[str, np.ndarray]], levels: Sequence[int], df: int):
        t = lambda a: torch.from_numpy(np.asarray(a, np.float32)).contiguous()  # noqa: E731
        pre = "vq3_d/~/structure_encoder"
        self.ne = (t(params[pre + "/init_node_embed"]["w"]), t(params[pre + "/init_node_embed"]["b"]))
        self.ee = (t(params[pre + "/init_edge_embed"]["w"]), t(params[pre + "/init_edge_embed"]["b"]))
        self.layers = []
        for l in range(3):
            m = f"{pre}/~/graph_neural_network/~/mpnn_layer" + ("" if l == 0 else f"_{l}")
            lin = lambda mod, i: (t(params[f"{m}/{mod}/~/linear_{i}"]["w"]), t(params[f"{m}/{mod}/~/linear_{i}"]["b"]))  # noqa: E731
            ln = lambda nm: (t(params[f"{m}/{nm}"]["scale"]), t(params[f"{m}/{nm}"]["offset"]))  # noqa: E731
            self.layers.append(dict(msg=[lin("node_mlp_0", i) for i in range(3)],
                                    ffn=[lin("node_mlp_1", i) for i in range(2)],
                                    edge=[lin("edge_mlp", i) for i in range(3)],
                                    ln=[ln("norm_msg"), ln("norm_msg_1"), ln("norm_msg_2")]))
        ds = "vq3_d/~/cross_attn_downsampling/cross_attn_scaler_iteration"
        ca, at = ds + "/cross_attention", ds + "/cross_attention/attention"
        self.blocks = []
        for b in range(3):
            g = lambda mod, nm: t(params[mod][nm][b])  # noqa: E731
            tr = lambda nm: (g(f"{ds}/{nm}/input_layer_norm", "scale"), g(f"{ds}/{nm}/input_layer_norm", "offset"),  # noqa: E731
                             g(f"{ds}/{nm}/transition1", "weights"), g(f"{ds}/{nm}/transition1", "bias"),
                             g(f"{ds}/{nm}/transition2", "weights"), g(f"{ds}/{nm}/transition2", "bias"))
            self.blocks.append(dict(
                qn=(g(ca + "/query_norm", "scale"), g(ca + "/query_norm", "offset")),
                dn=(g(ca + "/data_norm", "scale"), g(ca + "/data_norm", "offset")),
                wq=g(at, "query_w"), wk=g(at, "key_w"), wv=g(at, "value_w"), wg=g(at, "gating_w"),
                bg=g(at, "gating_b"), wo=g(at, "output_w"), bo=g(at, "output_b"),
                rt=tr("resampled_transition"), ot=tr("original_transition")))
        self.down = (t(params["vq3_d/down_proj"]["w"]), t(params["vq3_d/down_proj"]["b"]))
        self.levels = torch.tensor(list(levels), dtype=torch.float32)
        self.levels_i = torch.tensor(list(levels), dtype=torch.int64)
        self.df = df
        self.T = P_NODES // df
        L = self.levels_i
        self.basis = torch.cat([torch.ones(1, dtype=torch.int64), torch.cumprod(L[:-1], 0)])
        K = int(torch.prod(L))
        idx = torch.arange(K)[:, None]
        digits = torch.remainder(torch.div(idx, self.basis, rounding_mode="floor"), L)
        self.codebook = ((digits.float() - (L // 2).float()) / (L // 2).float()) * (L // 2).float()
        self.node_pe = _pe(torch.arange(P_NODES), P_NODES)
        self.tok_pe = _pe(torch.arange(self.T), self.T)
        tok = torch.arange(self.T)[:, None]
        node = torch.arange(P_NODES)[None, :]
        self.local = ((node >= tok * df) & (node < tok * df + df)).float()  # model.py:274-298

    @torch.no_grad()
    def forward(self, graphs) -> Dict[str, np.ndarray]:
        """graphs: padded ProteinGraph list (pst_amd.graph.pad_protein_graph) → numpy outputs
        shaped like the reference's QuantizerOutput [B, T, ...]."""
        B = len(graphs)
        snd = torch.from_numpy(np.stack([g.senders for g in graphs]))          # [B, E]
        rcv = torch.from_numpy(np.stack([g.receivers for g in graphs]))
        feat = torch.from_numpy(np.stack([g.edge_features for g in graphs]).astype(np.float32))
        nmask = torch.from_numpy(np.stack([g.nodes_mask for g in graphs]).astype(np.float32))   # [B,P,1]
        tmask = torch.from_numpy(np.stack([g.tokens_mask for g in graphs]).astype(np.float32))  # [B,T,1]
        # structure encoder: node PE table, per-edge PE of (sender - receiver)
        h = (self.node_pe @ self.ne[0] + self.ne[1]).expand(B, P_NODES, H)
        e = torch.cat([_pe(snd - rcv, P_NODES), feat], -1) @ self.ee[0] + self.ee[1]   # [B,E,128]
        bidx = torch.arange(B)[:, None]
        for L in self.layers:
            x = torch.cat([h[bidx, snd], h[bidx, rcv], e], -1)
            m = _gelu(x @ L["msg"][0][0] + L["msg"][0][1])
            m = _gelu(m @ L["msg"][1][0] + L["msg"][1][1])
            m = m @ L["msg"][2][0] + L["msg"][2][1]
            agg = torch.zeros(B, P_NODES, H).index_add_(1, rcv[0], m) if B == 1 else \
                torch.stack([torch.zeros(P_NODES, H).index_add_(0, rcv[i], m[i]) for i in range(B)])
            agg = agg / K_NB
            h = _masked_ln(h + agg, nmask, *L["ln"][0])
            f = _gelu(h @ L["ffn"][0][0] + L["ffn"][0][1]) @ L["ffn"][1][0] + L["ffn"][1][1]
            h = _masked_ln(h + f, nmask, *L["ln"][1])
            x = torch.cat([h[bidx, snd], h[bidx, rcv], e], -1)
            u = _gelu(x @ L["edge"][0][0] + L["edge"][0][1])
            u = _gelu(u @ L["edge"][1][0] + L["edge"][1][1])
            u = u @ L["edge"][2][0] + L["edge"][2][1]
            e = _masked_ln((e + u).reshape(B, -1, K_NB, H), nmask[:, :, None], *L["ln"][2]).reshape(B, -1, H)
        # cross-attention downsampler (3 blocks, dense over the 512 keys)
        mask = tmask * nmask.transpose(1, 2)                                    # [B,T,P]
        mask = (mask * self.local)[:, None].expand(B, 4, self.T, P_NODES)
        bias = 1e9 * (mask - 1.0)
        o = h
        r = self.tok_pe.expand(B, self.T, H)
        for bk in self.blocks:
            q_in = _ln(r, *bk["qn"])
            d_in = _ln(o, *bk["dn"])
            q = torch.einsum("bqa,ahc->bqhc", q_in, bk["wq"]) * 32 ** -0.5
            k = torch.einsum("bka,ahc->bkhc", d_in, bk["wk"])
            v = torch.einsum("bka,ahc->bkhc", d_in, bk["wv"])
            w = torch.softmax(torch.einsum("bqhc,bkhc->bhqk", q, k) + bias, -1)
            wa = torch.einsum("bhqk,bkhc->bqhc", w, v)
            wa = wa * torch.sigmoid(torch.einsum("bqc,chv->bqhv", q_in, bk["wg"]) + bk["bg"])
            r = r + torch.einsum("bqhc,hco->bqo", wa, bk["wo"]) + bk["bo"]
            for trn, which in ((bk["rt"], "r"), (bk["ot"], "o")):
                s, off, w1, b1, w2, b2 = trn
                a = torch.relu(_ln(r if which == "r" else o, s, off) @ w1 + b1) @ w2 + b2
                if which == "r":
                    r = r + a
                else:
                    o = o + a
        pre = r / (torch.linalg.vector_norm(r, dim=-1, keepdim=True) + 1e-6)
        z = pre @ self.down[0] + self.down[1]
        # FSQ (quantize.py:175-239)
        Lf = self.levels
        half_l = (Lf - 1) * (1 - 1e-3) / 2
        offset = torch.where(self.levels_i % 2 == 0, 0.5, 0.0)
        shift = torch.tan(offset / half_l)
        b = (torch.tanh(z + shift) * half_l - offset) * tmask
        qz = torch.round(b)
        hw = (self.levels_i // 2).float()
        idx = (((qz / hw) * hw + hw) * self.basis.float()).sum(-1).to(torch.int64)
        K = self.codebook.shape[0]
        onehot = torch.nn.functional.one_hot(idx, K).float() * tmask
        hist = onehot.reshape(-1, K).sum(0)
        avg = hist / hist.sum()
        perplexity = torch.exp(-torch.sum(avg * torch.log(avg + 1e-10)))
        sq = (b[..., None, :] - self.codebook[None, None]) ** 2                 # [B,T,K,D]
        distances = (tmask[..., None] * sq).sum(-1)
        soft = torch.softmax(sq.sum(-1), -1)
        return dict(tokens=idx.numpy().astype(np.uint32), bounded=b.numpy(), quantize=qz.numpy(),
                    pre_proj=pre.numpy(), distances=distances.numpy(), soft_proba=soft.numpy(),
                    perplexity=float(perplexity))


def padded_graphs(samples_pos_flags, df):
    """[(positions f64 [R,37,3], flags u8 [R,37])] → padded reference graphs, via the C oracle."""
    from pst_amd.graph import pad_protein_graph
    from . import oracle as O
    out = []
    for pos, fl in samples_pos_flags:
        g = O.graph(pos, fl)
        n = g["n"]
        out.append(pad_protein_graph(n, g["senders"].reshape(n, K_NB), g["feat"][:, :27].reshape(n, K_NB, 27),
                                     np.zeros((n, 3)), df))
    return out
