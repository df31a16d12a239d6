"""GPU parity: COO sparse x dense products of the outlier decomposition against
oracle/spmm.py (bit-exact: both follow the kernels' fp16 / fp32 accumulation order)."""
import numpy as np
import pytest
import torch

from oracle import spmm as ref_spmm

pytestmark = pytest.mark.gpu


def _F():
    import python_src_quants.functional as F
    return F


def _coo(rng, rows, cols, max_per_row, dev, shuffle=True):
    r, c = [], []
    for i in range(rows):
        k = int(rng.integers(0, max_per_row + 1))
        cs = rng.choice(cols, size=k, replace=False)
        r += [i] * k
        c += sorted(cs.tolist())
    r, c = np.array(r, np.int32), np.array(c, np.int32)
    v = (rng.standard_normal(r.size) * 3).astype(np.float16)
    if shuffle:
        p = rng.permutation(r.size)
        r, c, v = r[p], c[p], v[p]
    F = _F()
    return F.COOSparseTensor(rows, cols, int(r.size), torch.from_numpy(r).to(dev), torch.from_numpy(c).to(dev),
                             torch.from_numpy(v).to(dev)), (r, c, v)


@pytest.mark.parametrize("shape", [(64, 128, 1000), (7, 33, 4104), (300, 256, 64)])
def test_spmm_coo_very_sparse_fp16(dev, shape):
    F = _F()
    rows, k, n = shape
    rng = np.random.default_rng(rows * 7 + n)
    coo, (r, c, v) = _coo(rng, rows, k, 32, dev, shuffle=False)   # the wrapper's groups need row-sorted COO
    B = torch.from_numpy((rng.standard_normal((k, n)) * 0.5).astype(np.float16)).to(dev)
    out0 = torch.from_numpy((rng.standard_normal((rows, n))).astype(np.float16)).to(dev)
    got = F.spmm_coo_very_sparse(coo, B, out=out0.clone())
    exp = ref_spmm.spmm_coo_very_sparse(r, c, v, B.cpu().numpy(), out0.cpu().numpy())
    assert np.array_equal(got.cpu().numpy().view(np.uint16), exp.view(np.uint16))


@pytest.mark.parametrize("with_stats", [True, False])
def test_spmm_coo_very_sparse_int8(dev, with_stats):
    F = _F()
    rows, k, n = 40, 96, 2056
    rng = np.random.default_rng(5)
    coo, (r, c, v) = _coo(rng, rows, k, 20, dev, shuffle=False)
    Bn = rng.integers(-127, 128, size=(k, n)).astype(np.int8)
    Bn[:, :7] = 0
    B = torch.from_numpy(Bn).to(dev)
    stats = torch.from_numpy((rng.random(n) * 4 + 0.1).astype(np.float32)).to(dev) if with_stats else None
    got = F.spmm_coo_very_sparse(coo, B, dequant_stats=stats)
    exp = ref_spmm.spmm_coo_very_sparse(r, c, v, Bn, np.zeros((rows, n), np.float16),
                                         None if stats is None else stats.cpu().numpy())
    assert np.array_equal(got.cpu().numpy().view(np.uint16), exp.view(np.uint16))


@pytest.mark.parametrize("transposed", [False, True])
def test_spmm_coo(dev, transposed):
    F = _F()
    rows, k, n = 50, 200, 300
    rng = np.random.default_rng(11)
    coo, (r, c, v) = _coo(rng, rows, k, 40, dev, shuffle=True)
    Bn = (rng.standard_normal((k, n)) * 0.5).astype(np.float16)
    B = torch.from_numpy(Bn).to(dev)
    if transposed:
        B = B.t().contiguous().t()
    got = F.spmm_coo(coo, B)
    exp = ref_spmm.spmm_coo(r, c, v, rows, Bn)
    assert np.array_equal(got.cpu().numpy().view(np.uint16), exp.view(np.uint16))
    dense = torch.zeros(rows, k, dtype=torch.float32)
    dense[torch.from_numpy(r).long(), torch.from_numpy(c).long()] = torch.from_numpy(v.astype(np.float32))
    assert torch.allclose(got.float().cpu(), dense @ torch.from_numpy(Bn).float(), rtol=1e-2, atol=1e-2)
