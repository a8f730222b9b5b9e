"""GPU FSQ aux (pst_codebook_aux / _device) vs the oracle: distances and soft_proba bitwise,
argmin exact, histogram = bincount of the token ids, perplexity per quantize.py:211-224."""
import numpy as np
import pytest
import torch  # before libpst loads: torch's bundled HIP runtime must open the GPU first

from oracle import oracle as O
from pst_amd import params as P
from pst_amd import synthetic
from pst_amd._native import Tokenizer, pack_samples
from pst_amd.config import LEVELS

pytestmark = pytest.mark.gpu


def _run(cb, df, sizes, seed=77):
    tk = Tokenizer(0, cb, df, P.random_blob(len(LEVELS[cb]), seed))
    ss = [synthetic.synthetic_protein(n, 900 + i) for i, n in enumerate(sizes)]
    pos, flags, off = pack_samples(ss)
    tok, nt, nn = tk.tokenize_packed(pos, flags, off)
    R = int(off[-1])
    aux = tk.aux(R)
    rows = np.concatenate([np.arange(off[b], off[b] + nt[b]) for b in range(len(ss))])
    return tk, tok[rows], aux["bounded"][rows], int(nt.sum())


@pytest.mark.parametrize("cb,df,sizes", [(4096, 1, (51, 130, 64)), (64000, 4, (200, 77)), (432, 1, (60,)),
                                         (1728, 1, (90,)), (64000, 1, (120,))])
def test_codebook_aux_bitwise(cb, df, sizes):
    tk, tokens, bounded, T = _run(cb, df, sizes)
    got = tk.codebook_aux(T)
    want = O.fsq_aux(LEVELS[cb], bounded)
    assert np.array_equal(got["distances"].view(np.uint32), want["distances"].view(np.uint32))
    assert np.array_equal(got["soft_proba"].view(np.uint32), want["soft_proba"].view(np.uint32))
    assert np.array_equal(got["argmin"], want["argmin"])
    ppl, hist = O.perplexity(tokens, tk.codebook_size)
    assert np.array_equal(got["histogram"], hist)
    assert abs(got["perplexity"] - ppl) <= 1e-6 * ppl
    # FSQ rounding == nearest code away from exact .5 ties
    assert np.mean(got["argmin"] == tokens) > 0.999
    tk.close()


def test_codebook_aux_device_matches_host():
    tk, tokens, bounded, T = _run(4096, 2, (100, 256, 57))
    host = tk.codebook_aux(T)
    cap = (100 + 256 + 57) // 2 + 3
    dev = torch.device("cuda", 0)
    dd = torch.zeros((cap, 4096), dtype=torch.float32, device=dev)
    dp = torch.zeros((cap, 4096), dtype=torch.float32, device=dev)
    da = torch.zeros(cap, dtype=torch.int32, device=dev)
    dh = torch.zeros(4096, dtype=torch.int32, device=dev)
    tk.codebook_aux_device(dd.data_ptr(), dp.data_ptr(), da.data_ptr(), dh.data_ptr(), cap)
    tk.sync()
    assert np.array_equal(dd[:T].cpu().numpy(), host["distances"])
    assert np.array_equal(dp[:T].cpu().numpy(), host["soft_proba"])
    assert np.array_equal(da[:T].cpu().numpy().view(np.uint32), host["argmin"])
    assert np.array_equal(dh.cpu().numpy().view(np.uint32), host["histogram"])
    with pytest.raises(ValueError):
        tk.codebook_aux_device(dd.data_ptr(), 0, 0, 0, 10)
    tk.close()
