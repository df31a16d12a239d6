"""Autograd entry points of the quantized matmuls: LLM.int8 (`matmul` / MatMul8bitLt) and 4-bit (`matmul_4bit` /
MatMul4Bit), with the reference's call signatures, return shapes and gradients
(ref:python_src_quants/autograd/_functions.py:246-577).

The forward passes are built around this backend's kernels rather than the reference's call chain:

* int8 -- an inference forward (no outliers, no gradient) quantises the activations in ONE pass
  (F.int8_row_quant, rows only) and runs the fused igemmlt + mm_dequant kernel on the row-major int8 weight
  (F.igemmlt_dequant); the training / outlier forward keeps the reference's double_quant (rows and columns, plus the
  COO outliers above the threshold) and adds the fp16 outlier product.  A weight that only exists in a
  col_turing / col_ampere layout (a legacy checkpoint's CxB) goes through transform + igemmlt + mm_dequant.
* 4-bit -- functional.gemm_4bit for any number of rows (its own routing: multi-row GEMV, few-token kernel, fused
  kernel, or dequantise + the hand-written k_hgemm), replacing dequantize_4bit + F.linear (reference line 507); a
  single activation row without gradient takes the decode GEMV exactly as the reference routes it.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional
import warnings

import torch

from .. import functional as F
from ..functional import prod


@dataclass
class MatmulLtState:
    """Per-layer LLM.int8 state (the reference's field schema, ref:autograd/_functions.py:246-285).  On this backend
    CB (row-major int8 [out, in]) and SCB are what the forward multiplies; CxB / SB are honoured when a checkpoint
    supplies only the col_turing / col_ampere form."""
    _tile_indices: Optional[torch.Tensor] = None
    force_no_igemmlt: bool = False
    CB = None
    CxB = None
    SB = None
    SCB = None
    CxBt = None
    SBt = None
    CBt = None
    subB = None
    outlier_pool = None
    has_accumulated_gradients = False
    threshold = 0.0
    idx = None
    is_training = True
    has_fp16_weights = True
    memory_efficient_backward = False
    use_pool = False
    formatB = F.get_special_format_str()

    def reset_grads(self):
        self.CB = self.CxB = self.SB = self.SCB = None
        self.CxBt = self.SBt = self.CBt = None


def supports_igemmlt(device: torch.device) -> bool:
    return device.type == "cuda"


def _empty_forward(ctx, A, B, bias, weight_shape):
    """Zero-element input: remember the operands for backward, return an empty output of the matmul's shape (A's
    last dimension contracts with whichever weight dimension it matches)."""
    ctx.is_empty = True
    ctx.A, ctx.B, ctx.bias = A, B, bias
    tail = weight_shape[1:] if A.shape[-1] == weight_shape[0] else weight_shape[:1]
    return torch.empty(A.shape[:-1] + tail, dtype=A.dtype, device=A.device)


def _empty_backward(ctx):
    return (torch.zeros_like(ctx.A), torch.zeros_like(ctx.B), None,
            None if ctx.bias is None else torch.zeros_like(ctx.bias), None)


# ----------------------------------------------------------------------------- LLM.int8 pieces
def _quantize_activations(A2: torch.Tensor, state: MatmulLtState, for_backward: bool):
    """(CA, CAt, SCA, SCAt, coo) of the fp16 activations.  Without outliers or backward only the row half is needed,
    and the one-pass kernel produces it; otherwise double_quant (rows, columns and the COO outliers)."""
    A16 = A2.to(torch.float16)
    if state.threshold == 0.0 and not for_backward:
        CA, SCA = F.int8_row_quant(A16)
        return CA, None, SCA, None, None
    return F.double_quant(A16, threshold=state.threshold)


def _quantize_weight(B: torch.Tensor, state: MatmulLtState) -> torch.Tensor:
    """fp16-weight layers quantise B when training without an accumulated gradient, or the first time; returns the
    (contiguous) B used for the outlier columns."""
    if B.shape[0] == B.stride(1) and not B.is_contiguous():
        B = B.contiguous()
    first_time = state.CB is None and state.CxB is None
    accumulating = B.is_leaf and B.grad is not None
    if first_time or (state.is_training and not accumulating):
        state.reset_grads()
        state.CB, state.CBt, state.SCB, state.SCBt, _ = F.double_quant(B.to(torch.float16))
    return B


def _split_outliers(A2, B, CA, CAt, coo, state: MatmulLtState):
    """Columns of A holding an outlier (|a| > threshold) leave the int8 product: their int8 entries are zeroed and
    the fp16 sub-product A[:, idx] @ W[:, idx]^T is returned for the caller to add (subA, or None)."""
    if coo is None:
        return None
    if state.has_fp16_weights:
        idx = torch.unique(coo.colidx).long()
        state.subB = B[:, idx].t().contiguous()
    else:
        idx = torch.unique(coo.colidx).long()
        if state.CB is not None:
            cols = state.CB[:, idx].clone()
        else:
            cols = F.extract_outliers(state.CxB, state.SB, idx.int())
        state.subB = (cols * state.SCB.view(-1, 1) / 127.0).t().contiguous().to(A2.dtype)
    state.idx = idx
    CA[:, idx] = 0
    if CAt is not None:
        CAt[:, idx] = 0
    return A2[:, idx]


def _int8_product(A2, CA, SCA, state: MatmulLtState, bias, use_igemmlt: bool):
    """The dequantised int8 product in A's dtype, bias added (fused into the kernel's epilogue when it is fp16)."""
    fused = bias if bias is None or bias.dtype == torch.float16 else None
    if use_igemmlt and state.CB is not None:
        out = F.igemmlt_dequant(CA, state.CB, SCA, state.SCB, bias=fused)
    elif use_igemmlt:
        C32A, SA = F.transform(CA, "col32")
        out32, Sout32 = F.igemmlt(C32A, state.CxB, SA, state.SB)
        out = F.mm_dequant(out32, Sout32, SCA, state.SCB, bias=fused)
    else:     # no int8 GEMM on this device: the dequantised weight in A's dtype
        A_in = A2.clone()
        if state.idx is not None:
            A_in[:, state.idx.long()] = 0
        out = torch.nn.functional.linear(A_in, state.CB.to(A2.dtype)).mul_(state.SCB.unsqueeze(0).mul(1.0 / 127.0))
        fused = None
    out = out.to(A2.dtype)
    if bias is not None and fused is None:
        out = out.add_(bias)
    return out


def _dequantized_weight(state: MatmulLtState, dtype) -> torch.Tensor:
    """W ~ CB * SCB / 127 in `dtype` (for grad_A = grad @ W), from CB or from the col_turing / col_ampere CxB."""
    if state.CB is not None:
        CB = state.CB.to(dtype, copy=True)
    elif state.CxB is not None:
        CB, _ = F.transform(state.CxB, "row", state=state.SB)
        CB = CB.to(dtype)
    else:
        raise Exception("State must contain either CBt or CB or CxB matrix for backward")
    return CB.mul_(state.SCB.unsqueeze(1).mul(1.0 / 127.0))


class MatMul8bitLt(torch.autograd.Function):
    """LLM.int8 matmul out = A @ W^T: int8 activations x int8 weight with the dequantisation fused into the GEMM,
    plus the fp16 product of the outlier columns when a threshold is set."""

    @staticmethod
    def forward(ctx, A, B, out=None, bias=None, state=MatmulLtState):
        ctx.is_empty = False
        if prod(A.shape) == 0:
            return _empty_forward(ctx, A, B, bias, B.shape)
        if A.dtype != torch.float16:
            warnings.warn(f"MatMul8bitLt: inputs will be cast from {A.dtype} to float16 during quantization")
        in_shape = A.shape
        A2 = A.reshape(-1, A.shape[-1]) if A.dim() == 3 else A
        for_backward = any(ctx.needs_input_grad[:2])

        CA, CAt, SCA, SCAt, coo = _quantize_activations(A2, state, for_backward)
        if state.has_fp16_weights:
            B = _quantize_weight(B, state)
        subA = _split_outliers(A2, B, CA, CAt, coo, state)
        output = _int8_product(A2, CA, SCA, state, bias,
                               supports_igemmlt(A.device) and not state.force_no_igemmlt)
        if subA is not None:
            output += torch.matmul(subA, state.subB)

        n_out = state.SB[0][0] if state.SB else (state.CB.shape[0] if state.CB is not None else B.shape[0])
        ctx.state = state
        ctx.grad_shape = in_shape
        ctx.dtype_A, ctx.dtype_B, ctx.dtype_bias = A2.dtype, B.dtype, None if bias is None else bias.dtype
        if for_backward:
            ctx.tensors = (CAt, subA, A2)
            ctx.tensor_states = (SCAt, state.idx)
        else:
            ctx.tensors = [None, None, A2]
            ctx.tensor_states = (None, None)
            ctx.save_for_backward(None, None)
        if len(in_shape) == 3:
            return output.view(in_shape[0], in_shape[1], n_out).clone()
        return output.view(in_shape[0], n_out)

    @staticmethod
    def backward(ctx, grad_output):
        if ctx.is_empty:
            return _empty_backward(ctx)
        need_A, need_B, _, need_bias, _ = ctx.needs_input_grad
        CAt, subA, _A = ctx.tensors
        SCAt, idx = ctx.tensor_states
        state = ctx.state
        grad_bias = grad_output.sum(0, dtype=ctx.dtype_bias) if need_bias else None
        g2 = grad_output.reshape(-1, grad_output.shape[-1]).contiguous() if grad_output.dim() == 3 else grad_output
        Cg, Cgt, SCg, SCgt, _ = F.double_quant(g2.to(torch.float16))
        grad_B = grad_A = None
        if need_B:
            # grad_W[o, i] = sum_t g[t, o] A[t, i]: the int8 product over the token dimension, column-normalised
            grad_B = F.igemmlt_dequant(Cgt.t().contiguous(), CAt.t().contiguous(), SCgt, SCAt)
            if state.threshold > 0.0 and subA is not None:
                grad_B[:, idx] += torch.matmul(g2.t(), subA)
        if need_A:
            W = _dequantized_weight(state, ctx.dtype_A)
            grad_A = torch.matmul(g2.to(ctx.dtype_A), W).view(ctx.grad_shape).to(ctx.dtype_A)
        return grad_A, grad_B, None, grad_bias, None


# ----------------------------------------------------------------------------- 4-bit
def _weight_is_transposed_view(B: torch.Tensor) -> bool:
    """Linear4bit hands matmul_4bit `weight.t()` -- shape (1, n/2) over the packed storage (n/2, 1) -- meaning
    out = A @ W^T; the untransposed storage means out = A @ W (dequantize_4bit's rule, ref:functional.py:1420-1424)."""
    return B.shape[0] == 1


class MatMul4Bit(torch.autograd.Function):
    """4-bit weight matmul (ref:autograd/_functions.py:486-540): forward through functional.gemm_4bit for the
    A @ W^T orientation, dequantise + matmul otherwise; backward grad_A = grad @ dequantize_4bit(W)."""

    @staticmethod
    def forward(ctx, A, B, out=None, bias=None, quant_state: Optional[F.QuantState] = None):
        ctx.is_empty = False
        if prod(A.shape) == 0:
            return _empty_forward(ctx, A, B, bias, quant_state.shape)
        if _weight_is_transposed_view(B) and F.gemm_4bit_supported(A, quant_state):
            output = F.gemm_4bit(A, B, quant_state)
            if bias is not None:
                output = output + bias
        else:
            W = F.dequantize_4bit(B, quant_state).to(A.dtype)
            output = torch.nn.functional.linear(A, W.t(), bias)
        ctx.state = quant_state
        ctx.dtype_A, ctx.dtype_B, ctx.dtype_bias = A.dtype, B.dtype, None if bias is None else bias.dtype
        ctx.tensors = (None, B) if any(ctx.needs_input_grad[:2]) else (None, None)
        return output

    @staticmethod
    def backward(ctx, grad_output):
        if ctx.is_empty:
            return _empty_backward(ctx)
        need_A, _, _, need_bias, _ = ctx.needs_input_grad
        _, B = ctx.tensors
        grad_bias = grad_output.sum(0, dtype=ctx.dtype_bias) if need_bias else None
        grad_A = None
        if need_A:
            grad_A = torch.matmul(grad_output, F.dequantize_4bit(B, ctx.state).to(grad_output.dtype).t())
        return grad_A, None, None, grad_bias, None


def matmul(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None,
           state: Optional[MatmulLtState] = None, threshold=0.0, bias=None):
    """LLM.int8 out = A @ B^T (ref:autograd/_functions.py:543-554)."""
    state = state or MatmulLtState()
    if threshold > 0.0:
        state.threshold = threshold
    return MatMul8bitLt.apply(A, B, out, bias, state)


def matmul_4bit(A: torch.Tensor, B: torch.Tensor, quant_state: F.QuantState, out: Optional[torch.Tensor] = None,
                bias=None):
    """4-bit matmul with the reference's routing (ref:autograd/_functions.py:557-577): a single activation row
    without gradient goes to gemv_4bit(A, B.t()) -- whichever orientation B is given in, as the reference does
    (gemv_4bit reads the weight's shape from quant_state and computes A @ W^T; an A whose width is not W's in-features
    is rejected there); a hidden size that is not a multiple of the blocksize warns and takes MatMul4Bit."""
    assert quant_state is not None
    single_row = A.numel() == A.shape[-1] and not A.requires_grad
    if not single_row:
        return MatMul4Bit.apply(A, B, out, bias, quant_state)
    if A.shape[-1] % quant_state.blocksize != 0:
        warnings.warn(
            f"Some matrices hidden dimension is not a multiple of {quant_state.blocksize} and efficient inference "
            f"kernels are not supported for these (slow). Matrix input size found: {A.shape}",
        )
        return MatMul4Bit.apply(A, B, out, bias, quant_state)
    if A.shape[-1] != quant_state.shape[1]:
        raise ValueError(f"matmul_4bit: a single activation row of width {A.shape[-1]} against a weight of "
                         f"in_features {quant_state.shape[1]} (the decode GEMV computes A @ W^T)")
    out = F.gemv_4bit(A, B.t(), out, state=quant_state)
    if bias is not None:
        out += bias
    return out
