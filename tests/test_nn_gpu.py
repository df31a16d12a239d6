"""nn layers on the GPU: Linear4bit / Params4bit (A9), Linear8bitLt / Int8Params (A15) and their serialisation
(§8(f) row 1).

* Linear4bit forward on every route matmul_4bit takes (1 row -> GEMV kernel; 2..32 rows -> few-token kernel;
  more -> tile kernels; 3-D inputs), against F.linear with the dequantised weight, at the reference test's bound
  mean|d| < 0.115 (ref:tests_pvc/autograd.py:388-391) and the GEMM tolerance of BASELINE.md §5.
* Serialisation: Linear4bit.state_dict() (ref:nn/modules.py:436-445) -> torch.save -> torch.load(weights_only=True)
  -> Params4bit.from_prequantized (ref:nn/modules.py:271-289, QuantState.from_dict ref:functional.py:686-735) ->
  a forward bit-identical to the original layer's, nested and plain statistics, nf4 and fp4.
* Linear8bitLt: SCB + weight_format round trip (ref:nn/modules.py:725-811), including checkpoints whose weight is
  stored in the col32 / col_turing / col_ampere tile formats (un-tiled at load, ref:nn/modules.py:635-654)."""
import io

import pytest
import torch

pytestmark = pytest.mark.gpu


def _bnb():
    import python_src_quants as bnb
    return bnb


def _roundtrip(obj):
    buf = io.BytesIO()
    torch.save(obj, buf)
    buf.seek(0)
    return torch.load(buf, weights_only=True)


def _reference_out(x, layer):
    F = _bnb().functional
    W = F.dequantize_4bit(layer.weight.data, layer.weight.quant_state).float()
    y = torch.nn.functional.linear(x.float(), W)
    if layer.bias is not None:
        y = y + layer.bias.float()
    return y


@pytest.mark.parametrize("quant_type", ["nf4", "fp4"])
@pytest.mark.parametrize("compress_statistics", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("bias", [True, False])
def test_linear4bit_routes(dev, quant_type, compress_statistics, dtype, bias):
    bnb = _bnb()
    torch.manual_seed(1)
    K, N = 1024, 768
    layer = bnb.nn.Linear4bit(K, N, bias=bias, compute_dtype=dtype, compress_statistics=compress_statistics,
                              quant_type=quant_type)
    assert isinstance(layer.weight, bnb.nn.Params4bit) and not layer.weight.bnb_quantized
    layer = layer.to(dtype).cuda(dev)
    assert layer.weight.bnb_quantized and layer.weight.dtype == torch.uint8
    assert layer.weight.shape == (N * K // 2, 1)
    st = layer.weight.quant_state
    assert st.shape == (N, K) and st.nested == compress_statistics and st.quant_type == quant_type
    for shape in [(1, K), (1, 1, K), (7, K), (32, K), (300, K), (2, 150, K)]:
        x = torch.randn(*shape, device=dev, dtype=dtype)
        y = layer(x)
        assert y.shape == (*shape[:-1], N) and y.dtype == dtype
        ref = _reference_out(x, layer)
        err = (y.float() - ref).abs()
        rms = ref.pow(2).mean().sqrt().item()
        tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
        assert err.mean().item() < 0.115
        assert (err <= tol * rms + tol * ref.abs()).all(), (shape, err.max().item())


def test_linear4bit_fp32_input_and_grad(dev):
    """fp32 activations take the dequantise + matmul path; grads flow to the input (MatMul4Bit.backward,
    ref:autograd/_functions.py:520-540) and agree with the dequantised-weight reference."""
    bnb = _bnb()
    torch.manual_seed(2)
    layer = bnb.nn.LinearNF4(256, 128, bias=True).cuda(dev)
    x = torch.randn(9, 256, device=dev, requires_grad=True)
    y = layer(x)
    assert y.dtype == torch.float32
    x2 = x.detach().clone().requires_grad_(True)
    ref = _reference_out(x2, layer)
    torch.testing.assert_close(y, ref, atol=1e-4, rtol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g)
    torch.testing.assert_close(x.grad, x2.grad, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("quant_type", ["nf4", "fp4"])
@pytest.mark.parametrize("compress_statistics", [True, False])
def test_linear4bit_state_dict_roundtrip(dev, quant_type, compress_statistics):
    bnb = _bnb()
    torch.manual_seed(3)
    K, N = 2048, 512
    layer = bnb.nn.Linear4bit(K, N, bias=True, compute_dtype=torch.bfloat16, compress_statistics=compress_statistics,
                              quant_type=quant_type).to(torch.bfloat16).cuda(dev)
    sd = layer.state_dict()
    qs_key = f"weight.quant_state.bitsandbytes__{quant_type}"
    assert qs_key in sd and sd[qs_key].dtype == torch.uint8
    assert ("weight.nested_absmax" in sd) == compress_statistics
    loaded = _roundtrip({k: v.cpu() for k, v in sd.items()})
    # the HF-style reload: a fresh layer whose weight is rebuilt from the packed bytes + serialised state
    fresh = bnb.nn.Linear4bit(K, N, bias=True, compute_dtype=torch.bfloat16, quant_type=quant_type)
    stats = {k[len("weight."):]: v for k, v in loaded.items() if k.startswith("weight.")}
    fresh.weight = bnb.nn.Params4bit.from_prequantized(loaded["weight"], stats, device=dev)
    fresh.bias = torch.nn.Parameter(loaded["bias"].to(dev))
    assert fresh.weight.quant_state == layer.weight.quant_state
    assert torch.equal(fresh.weight.data, layer.weight.data)
    for rows in (1, 5, 64, 2048):
        x = torch.randn(rows, K, device=dev, dtype=torch.bfloat16)
        assert torch.equal(fresh(x), layer(x)), rows
    # pickling / deepcopy keep the quantised state
    import copy
    dup = copy.deepcopy(layer.weight)
    assert torch.equal(dup.data, layer.weight.data) and dup.quant_state == layer.weight.quant_state


def _int8_layer(dev, K, N, threshold=0.0, seed=4):
    bnb = _bnb()
    torch.manual_seed(seed)
    layer = bnb.nn.Linear8bitLt(K, N, bias=True, has_fp16_weights=False, threshold=threshold)
    w_fp16 = layer.weight.data.clone().half()
    layer = layer.cuda(dev)
    return layer, w_fp16


@pytest.mark.parametrize("threshold", [0.0, 6.0])
def test_linear8bitlt_forward_contract(dev, threshold):
    """Linear8bitLt vs the fp16 linear at the reference's matmullt bounds (ref:tests_pvc/autograd.py:277-280)."""
    K, N = 1024, 512
    layer, w = _int8_layer(dev, K, N, threshold)
    x = torch.randn(64, K, device=dev, dtype=torch.float16)
    if threshold > 0:
        x[:, torch.randint(0, K, (8,))] = 8.0
    y = layer(x)
    ref = torch.nn.functional.linear(x.float(), w.float().to(dev), layer.bias.float())
    n = y.numel()
    assert (~torch.isclose(y.float(), ref, atol=0.01, rtol=0.1)).sum().item() <= n * 0.0175
    assert (~torch.isclose(y.float(), ref, atol=0.035, rtol=0.2)).sum().item() <= n * 0.001


def test_linear8bitlt_state_dict_roundtrip(dev):
    bnb = _bnb()
    K, N = 768, 320
    layer, _ = _int8_layer(dev, K, N)
    x = torch.randn(33, K, device=dev, dtype=torch.float16)
    y0 = layer(x)                                   # moves CB/SCB into the matmul state
    sd = layer.state_dict()
    assert sd["weight"].dtype == torch.int8 and "SCB" in sd and int(sd["weight_format"]) == 0
    loaded = _roundtrip({k: v.cpu() for k, v in sd.items()})
    fresh = bnb.nn.Linear8bitLt(K, N, bias=True, has_fp16_weights=False)
    with pytest.raises(RuntimeError):
        fresh.load_state_dict(loaded)               # must be quantised (.cuda()) before loading SCB
    fresh = bnb.nn.Linear8bitLt(K, N, bias=True, has_fp16_weights=False).cuda(dev)
    fresh.load_state_dict(loaded)
    assert torch.equal(fresh(x), y0)


@pytest.mark.parametrize("fmt", ["col32", "col_turing", "col_ampere"])
@pytest.mark.parametrize("shape", [(320, 768), (100, 200)])
def test_linear8bitlt_tiled_checkpoint(dev, fmt, shape):
    """A checkpoint whose int8 weight is stored tiled (weight_format 1/2/3, padded tile shape) loads into the
    row-major layout and gives the row-major checkpoint's forward bit for bit."""
    bnb = _bnb()
    F = bnb.functional
    from python_src_quants.utils import LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING
    N, K = shape
    layer, _ = _int8_layer(dev, K, N, seed=5)
    x = torch.randn(17, K, device=dev, dtype=torch.float16)
    y0 = layer(x)
    sd = {k: v.clone() for k, v in layer.state_dict().items()}
    tiled, _ = F.transform(sd["weight"].to(dev).contiguous(), fmt)
    sd["weight"] = tiled.cpu()
    sd["weight_format"] = torch.tensor(LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING[fmt], dtype=torch.uint8)
    fresh = bnb.nn.Linear8bitLt(K, N, bias=True, has_fp16_weights=False).cuda(dev)
    fresh.load_state_dict(_roundtrip(sd))
    assert torch.equal(fresh(x), y0)
    with pytest.raises(ValueError):
        bad = dict(sd)
        bad["weight_format"] = torch.tensor(9, dtype=torch.uint8)
        bnb.nn.Linear8bitLt(K, N, bias=True, has_fp16_weights=False).cuda(dev).load_state_dict(bad)
