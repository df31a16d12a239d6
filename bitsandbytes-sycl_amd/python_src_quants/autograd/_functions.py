"""Autograd glue for the 4-bit and LLM.int8 matmuls
(mirrors ref:python_src_quants/autograd/_functions.py:246-577)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional
import warnings

import torch

from .. import functional as F
from ..functional import prod


@dataclass
class MatmulLtState:
    """ref:autograd/_functions.py:246-285.  On this backend the weight stays row-major int8
    (CB) and the forward runs the fused row-major igemmlt + mm_dequant kernel; a col_turing /
    col_ampere CxB (e.g. from a checkpoint) is still honoured through F.igemmlt."""
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
        self.CB = None
        self.CxB = None
        self.SB = None
        self.SCB = None
        self.CxBt = None
        self.SBt = None
        self.CBt = None


def supports_igemmlt(device: torch.device) -> bool:
    return device.type == "cuda"


class MatMul8bitLt(torch.autograd.Function):
    """LLM.int8 matmul: double_quant(A) -> int8 GEMM -> dequant (+ outlier fp16 matmul)."""

    @staticmethod
    def forward(ctx, A, B, out=None, bias=None, state=MatmulLtState):
        using_igemmlt = supports_igemmlt(A.device) and not state.force_no_igemmlt
        ctx.is_empty = False
        if prod(A.shape) == 0:
            ctx.is_empty = True
            ctx.A, ctx.B, ctx.bias = A, B, bias
            if A.shape[-1] == B.shape[0]:
                return torch.empty(A.shape[:-1] + B.shape[1:], dtype=A.dtype, device=A.device)
            return torch.empty(A.shape[:-1] + B.shape[:1], dtype=A.dtype, device=A.device)

        input_shape = A.shape
        if A.dtype != torch.float16:
            warnings.warn(f"MatMul8bitLt: inputs will be cast from {A.dtype} to float16 during quantization")
        if len(A.shape) == 3:
            A = A.reshape(-1, A.shape[-1])
        # 1. quantise A (row- and column-normalised; only the row half, in one pass over A, when there are
        #    no outliers to split off and no backward will read CAt)
        if state.threshold == 0.0 and not any(ctx.needs_input_grad[:2]):
            CA, SCA = F.int8_row_quant(A.to(torch.float16))
            CAt, SCAt, coo_tensorA = None, None, None
        else:
            CA, CAt, SCA, SCAt, coo_tensorA = F.double_quant(A.to(torch.float16), threshold=state.threshold)
        subA = None
        if state.threshold > 0.0 and coo_tensorA is not None and state.has_fp16_weights:
            idx = torch.unique(coo_tensorA.colidx).long()
            CA[:, idx] = 0
            CAt[:, idx] = 0
            subA = A[:, idx]
            state.subB = B[:, idx].t().contiguous()
            state.idx = idx
        # 2. quantise B (once, unless training fp16 weights)
        if state.has_fp16_weights:
            has_grad = B.is_leaf and B.grad is not None
            is_transposed = not B.is_contiguous() and B.shape[0] == B.stride(1)
            if is_transposed:
                B = B.contiguous()
            if (state.is_training and not has_grad) or (state.CB is None and state.CxB is None):
                state.reset_grads()
                CB, state.CBt, state.SCB, state.SCBt, _ = F.double_quant(B.to(torch.float16))
                state.CB = CB
        if coo_tensorA is not None and not state.has_fp16_weights:
            state.idx = torch.unique(coo_tensorA.colidx)
            if state.CB is not None:
                outliers = state.CB[:, state.idx.long()].clone()
            else:
                outliers = F.extract_outliers(state.CxB, state.SB, state.idx.int())
            state.subB = (outliers * state.SCB.view(-1, 1) / 127.0).t().contiguous().to(A.dtype)
            CA[:, state.idx.long()] = 0
            CAt[:, state.idx.long()] = 0
            subA = A[:, state.idx.long()]

        shapeB = state.SB[0] if state.SB else (state.CB.shape if state.CB is not None else B.shape)
        output_shape = (input_shape[0], input_shape[1], shapeB[0]) if len(input_shape) == 3 else (input_shape[0], shapeB[0])

        # 3. int8 matmul with the dequant fused in (bias fused when it is fp16)
        fused_bias = bias if (bias is None or bias.dtype == torch.float16) else None
        if using_igemmlt and state.CB is not None:
            output = F.igemmlt_dequant(CA, state.CB, SCA, state.SCB, bias=fused_bias)
        elif using_igemmlt:
            C32A, SA = F.transform(CA, "col32")
            out32, Sout32 = F.igemmlt(C32A, state.CxB, SA, state.SB)
            output = F.mm_dequant(out32, Sout32, SCA, state.SCB, bias=fused_bias)
        else:
            A_wo = A.clone()
            if state.idx is not None:
                A_wo[:, state.idx.long()] = 0
            output = torch.nn.functional.linear(A_wo, state.CB.to(A.dtype)).mul_(state.SCB.unsqueeze(0).mul(1.0 / 127.0))
            fused_bias = None
        output = output.to(A.dtype)
        if bias is not None and fused_bias is None:
            output = output.add_(bias)
        # 4. mixed-precision outlier matmul
        if coo_tensorA is not None and subA is not None:
            output += torch.matmul(subA, state.subB)

        ctx.state = state
        ctx.grad_shape = input_shape
        ctx.dtype_A, ctx.dtype_B, ctx.dtype_bias = A.dtype, B.dtype, None if bias is None else bias.dtype
        if any(ctx.needs_input_grad[:2]):
            ctx.tensors = (CAt, subA, A)
            ctx.tensor_states = (SCAt, state.idx)
        else:
            ctx.tensors = [None, None, A]
            ctx.tensor_states = (None, None)
            ctx.save_for_backward(None, None)
        clone_func = torch.clone if len(output_shape) == 3 else (lambda x: x)
        return clone_func(output.view(output_shape))

    @staticmethod
    def backward(ctx, grad_output):
        if ctx.is_empty:
            bias_grad = None if ctx.bias is None else torch.zeros_like(ctx.bias)
            return torch.zeros_like(ctx.A), torch.zeros_like(ctx.B), None, bias_grad, None
        req_gradA, req_gradB, _, req_gradBias, _ = ctx.needs_input_grad
        CAt, subA, A = ctx.tensors
        SCAt, idx = ctx.tensor_states
        state = ctx.state
        grad_A = grad_B = grad_bias = None
        if req_gradBias:
            grad_bias = grad_output.sum(0, dtype=ctx.dtype_bias)
        if len(grad_output.shape) == 3:
            grad_output = grad_output.reshape(-1, grad_output.shape[-1]).contiguous()
        Cgrad, Cgradt, SCgrad, SCgradt, _ = F.double_quant(grad_output.to(torch.float16))
        if req_gradB:
            # grad_B[o, i] = sum_t grad[t, o] * A[t, i]: int8 GEMM over the token dim (column-normalised)
            grad_B = F.igemmlt_dequant(Cgradt.t().contiguous(), CAt.t().contiguous(), SCgradt, SCAt)
            if state.threshold > 0.0 and subA is not None:
                grad_B[:, idx] += torch.matmul(grad_output.t(), subA)
        if req_gradA:
            if state.CB is not None:
                CB = state.CB.to(ctx.dtype_A, copy=True).mul_(state.SCB.unsqueeze(1).mul(1.0 / 127.0))
                grad_A = torch.matmul(grad_output.to(ctx.dtype_A), CB).view(ctx.grad_shape).to(ctx.dtype_A)
            elif state.CxB is not None:
                CB, _ = F.transform(state.CxB, "row", state=state.SB)
                CB = CB.to(ctx.dtype_A).mul_(state.SCB.unsqueeze(1).mul(1.0 / 127.0))
                grad_A = torch.matmul(grad_output.to(ctx.dtype_A), CB).view(ctx.grad_shape).to(ctx.dtype_A)
            else:
                raise Exception("State must contain either CBt or CB or CxB matrix for backward")
        return grad_A, grad_B, None, grad_bias, None


class MatMul4Bit(torch.autograd.Function):
    """4-bit weight matmul for M > 1 (ref:autograd/_functions.py:486-540).  Forward runs the fused
    NF4/FP4 GEMM kernel (dequantise tiles in LDS + MFMA) instead of dequantize_4bit + F.linear."""

    @staticmethod
    def forward(ctx, A, B, out=None, bias=None, quant_state: Optional[F.QuantState] = None):
        ctx.is_empty = False
        if prod(A.shape) == 0:
            ctx.is_empty = True
            ctx.A, ctx.B, ctx.bias = A, B, bias
            B_shape = quant_state.shape
            if A.shape[-1] == B_shape[0]:
                return torch.empty(A.shape[:-1] + B_shape[1:], dtype=A.dtype, device=A.device)
            return torch.empty(A.shape[:-1] + B_shape[:1], dtype=A.dtype, device=A.device)
        # B as the reference passes it: the transposed view of the packed weight (Linear4bit's weight.t(),
        # shape (1, n/2)) means out = A @ W^T with W [shape[0], shape[1]] -- the fused GEMM's orientation; the
        # untransposed storage (shape (n/2, 1)) means out = A @ W (dequantize_4bit's is_transposed rule,
        # ref:functional.py:1420-1424), which takes the dequantise + matmul path
        if B.shape[0] == 1 and F.gemm_4bit_supported(A, quant_state):
            output = F.gemm_4bit(A, B, quant_state)
            if bias is not None:
                output = output + bias
        else:
            output = torch.nn.functional.linear(A, F.dequantize_4bit(B, quant_state).to(A.dtype).t(), bias)
        ctx.state = quant_state
        ctx.dtype_A, ctx.dtype_B, ctx.dtype_bias = A.dtype, B.dtype, None if bias is None else bias.dtype
        ctx.tensors = (None, B) if any(ctx.needs_input_grad[:2]) else (None, None)
        return output

    @staticmethod
    def backward(ctx, grad_output):
        if ctx.is_empty:
            bias_grad = None if ctx.bias is None else torch.zeros_like(ctx.bias)
            return torch.zeros_like(ctx.A), torch.zeros_like(ctx.B), None, bias_grad, None
        req_gradA, _, _, req_gradBias, _ = ctx.needs_input_grad
        _, B = ctx.tensors
        grad_A, grad_B, grad_bias = None, None, None
        if req_gradBias:
            grad_bias = grad_output.sum(0, dtype=ctx.dtype_bias)
        if req_gradA:
            grad_A = torch.matmul(grad_output, F.dequantize_4bit(B, ctx.state).to(grad_output.dtype).t())
        return grad_A, grad_B, None, grad_bias, None


def matmul(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None,
           state: Optional[MatmulLtState] = None, threshold=0.0, bias=None):
    state = state or MatmulLtState()
    if threshold > 0.0:
        state.threshold = threshold
    return MatMul8bitLt.apply(A, B, out, bias, state)


def matmul_4bit(A: torch.Tensor, B: torch.Tensor, quant_state: F.QuantState, out: Optional[torch.Tensor] = None,
                bias=None):
    """Routing of ref:autograd/_functions.py:557-577: one activation row without grad -> gemv_4bit."""
    assert quant_state is not None
    if A.numel() == A.shape[-1] and A.requires_grad is False and B.shape[0] == 1:
        if A.shape[-1] % quant_state.blocksize != 0:
            warnings.warn(
                f"Some matrices hidden dimension is not a multiple of {quant_state.blocksize} and efficient inference "
                f"kernels are not supported for these (slow). Matrix input size found: {A.shape}",
            )
            return MatMul4Bit.apply(A, B, out, bias, quant_state)
        out = F.gemv_4bit(A, B.t(), out, state=quant_state)
        if bias is not None:
            out += bias
        return out
    return MatMul4Bit.apply(A, B, out, bias, quant_state)
