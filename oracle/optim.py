"""numpy restatement of the reference's optimizer updates (TEST INFRASTRUCTURE ONLY; see
oracle/__init__.py for who may import this).

  8-bit blockwise, 2 states (Adam)   ref:sycl/sycl_code/kernel_quant.cpp:2715-2972
  8-bit blockwise, 1 state           ref:sycl/sycl_code/kernel_quant.cpp:2977-3208
  32-bit, 2 / 1 states               ref:sycl/sycl_code/kernel_quant.cpp:1614-1760, 1884-2060
  launch constants                   ref:sycl/sycl_code/op_quant.cpp:1135-1138 (2048-element blocks)

Every fp32 operation of the reference is one numpy float32 operation here, in the reference's
order.  Intended semantics where the reference is defective:
  Q21 quantize_2D (kernel_quant.cpp:840-888) replaces the code lookup of every search step after the
      first by 0; the intended search is the upstream one, which equals dQuantize<0>
      (ref.quantize_8bit_dynamic) for maps with code[255] == 1 (both dynamic maps);
  Q22 the 1-state kernel switches on case labels 1/2/3/4 while the enum (ops.h:68-76) gives
      MOMENTUM 1, RMSPROP 2, ADAGRAD 4, LION 5: the intended update per optimizer is used;
  Q23 the last block's tail is loaded as upstream's defaults (g 0, state1 code 128, state2 code 0).
Parity of this file is pinned by the reference source only (no reference run); the
reference's own test (tests_pvc/test_optimizer8bit.py) bounds the result against torch.optim.
"""
from __future__ import annotations

import math

import numpy as np

from .ref import F32, FLT_MAX, as_f32, cast_out, quantize_8bit_dynamic

BLOCK = 2048
ADAM, MOMENTUM, RMSPROP, LARS, ADAGRAD, LION = 0, 1, 2, 3, 4, 5
NAME2OPT = {"adam": ADAM, "momentum": MOMENTUM, "rmsprop": RMSPROP, "adagrad": ADAGRAD, "lion": LION}


def scalars(beta1, beta2, eps, step, lr, weight_decay):
    """Host-side constants: pow(float, int) promotes to double in the reference (kernel_quant.cpp:2740-2742)."""
    b1, b2 = float(F32(beta1)), float(F32(beta2))
    c1 = F32(1.0 - math.pow(b1, float(step)))
    c2 = F32(math.sqrt(1.0 - math.pow(b2, float(step))))
    lr, eps, wd = F32(lr), F32(eps), F32(weight_decay)
    step_size = F32(F32(-lr * c2) / c1)
    return {"step_size": step_size, "c2eps": F32(c2 * eps), "decay": F32(F32(1.0) - F32(lr * wd))}


def _t(v, dtype):
    """fp32 -> T -> fp32 (one RNE cast), as an assignment to a T variable in the reference."""
    return as_f32(cast_out(np.asarray(v, F32), dtype), dtype)


def _sgn(x):
    return ((x > 0).astype(F32) - (x < 0).astype(F32)).astype(F32)


def _requant(code, s, absmax_per_elem, signed):
    with np.errstate(divide="ignore", invalid="ignore"):
        x = (s / absmax_per_elem).astype(F32)
    c = quantize_8bit_dynamic(code, x).astype(np.int64)
    if signed:   # keep the sign of the state (kernel_quant.cpp:2933-2941)
        flip = np.signbit(code[c]) != np.signbit(s)
        c = np.where(flip, np.where(s > 0, c + 1, c - 1), c) & 0xFF
    return c.astype(np.uint8)


def _pad(a, n_full, fill):
    out = np.full(n_full, fill, dtype=a.dtype)
    out[:a.size] = a
    return out


def update_8bit_blockwise(name, g, p, c1, c2, code1, code2, absmax1, absmax2, beta1, beta2, eps, step, lr,
                          weight_decay=0.0, gnorm_scale=1.0, skip_zeros=False, dtype="fp32"):
    """One step.  g, p: arrays in `dtype` storage (bf16 as uint16 bits); c1, c2: uint8 codes; absmax*:
    fp32 per 2048-block.  Returns (p_new in `dtype` storage, c1, c2, absmax1, absmax2)."""
    opt = NAME2OPT[name]
    n = g.size
    nb = (n + BLOCK - 1) // BLOCK
    nf = nb * BLOCK
    k = scalars(beta1, beta2, eps, step, lr, weight_decay)
    b1, b2, eps, lr, wd, gsc = F32(beta1), F32(beta2), F32(eps), F32(lr), F32(weight_decay), F32(gnorm_scale)
    one = F32(1.0)
    code1 = np.asarray(code1, F32)
    gv = _pad(as_f32(g.reshape(-1), dtype), nf, F32(0))
    pv = _pad(as_f32(p.reshape(-1), dtype), nf, F32(0))
    q1 = _pad(c1.reshape(-1).astype(np.int64), nf, 128)
    blk = np.arange(nf) // BLOCK
    am1 = np.asarray(absmax1, F32)[blk]
    with np.errstate(over="ignore", invalid="ignore"):
        if opt == ADAM:
            code2 = np.asarray(code2, F32)
            q2 = _pad(c2.reshape(-1).astype(np.int64), nf, 0)
            am2 = np.asarray(absmax2, F32)[blk]
            ok = np.isfinite(gv)
            gs = (gv * gsc).astype(F32)
            s2 = (code2[q2] * am2).astype(F32)
            s2 = (s2 * b2 + ((one - b2) * gs).astype(F32) * gs).astype(F32)
            s1 = (code1[q1] * am1).astype(F32)
            s1 = (s1 * b1 + ((one - b1) * gs).astype(F32)).astype(F32)
            s1 = np.where(ok, s1, F32(0))
            s2 = np.where(ok, s2, F32(0))
            m1 = np.fmax.reduce(np.abs(s1).reshape(nb, BLOCK), axis=1, initial=-FLT_MAX).astype(F32)
            m2 = np.fmax.reduce(np.abs(s2).reshape(nb, BLOCK), axis=1, initial=-FLT_MAX).astype(F32)
            upd = (k["step_size"] * (s1 / (np.sqrt(s2).astype(F32) + k["c2eps"]).astype(F32)).astype(F32)).astype(F32)
            pn = _t((pv + upd).astype(F32), dtype)
            if wd > 0:
                pn = _t((pn * k["decay"]).astype(F32), dtype)
            pn = np.where(ok, pn, _t(pv, dtype))
            n1 = _requant(code1, s1, m1[blk], True)
            n2 = _requant(code2, s2, m2[blk], False)
            return cast_out(pn[:n], dtype), n1[:n], n2[:n], m1, m2
        gs = (gv * gsc).astype(F32)
        upd_mask = np.ones(nf, bool) if not skip_zeros else (gv != 0)
        s_old = (code1[q1] * am1).astype(F32)
        s1 = s_old.copy()
        gl = gv.copy()
        if wd > 0:
            if opt == LION:
                pv = np.where(upd_mask, _t((pv * k["decay"]).astype(F32), dtype), pv)
            else:
                gs = np.where(upd_mask, (gs + (pv * wd).astype(F32)).astype(F32), gs)
        if opt == MOMENTUM:
            new = gs if step == 1 else (s_old * b1 + gs).astype(F32)
        elif opt == LION:
            t = (s_old * b1 + ((one - b1) * gs).astype(F32)).astype(F32)
            gl = np.where(upd_mask, _t((lr * _sgn(t)).astype(F32), dtype), gl)
            new = (s_old * b2 + ((one - b2) * gs).astype(F32)).astype(F32)
        elif opt == RMSPROP:
            new = (s_old * b1 + ((one - b1) * (gs * gs).astype(F32)).astype(F32)).astype(F32)
        else:
            new = (s_old + (gs * gs).astype(F32)).astype(F32)
        s1 = np.where(upd_mask, new, s_old).astype(F32)
        m1 = np.fmax.reduce(np.abs(s1).reshape(nb, BLOCK), axis=1, initial=-FLT_MAX).astype(F32)
        if opt == MOMENTUM:
            pn = (pv - (lr * s1).astype(F32)).astype(F32)
        elif opt == LION:
            pn = (pv - gl).astype(F32)
        else:
            pn = (pv - (lr * (gl / (np.sqrt(s1).astype(F32) + eps).astype(F32)).astype(F32)).astype(F32)).astype(F32)
        pn = np.where(upd_mask, pn, pv)
        n1 = _requant(code1, s1, m1[blk], True)
        return cast_out(pn[:n], dtype), n1[:n], None, m1, None


def update_32bit(name, g, p, s1, s2, beta1, beta2, eps, step, lr, weight_decay=0.0, gnorm_scale=1.0,
                 skip_zeros=False, dtype="fp32"):
    """kOptimizer32bit{2,1}State with max_unorm = 0.  Returns (p_new in `dtype` storage, s1, s2)."""
    opt = NAME2OPT[name]
    k = scalars(beta1, beta2, eps, step, lr, weight_decay)
    b1, b2, eps, lr, wd, gsc = F32(beta1), F32(beta2), F32(eps), F32(lr), F32(weight_decay), F32(gnorm_scale)
    one = F32(1.0)
    gv = as_f32(g.reshape(-1), dtype)
    pv = as_f32(p.reshape(-1), dtype)
    s1 = np.asarray(s1, F32).reshape(-1).copy()
    s2 = None if s2 is None else np.asarray(s2, F32).reshape(-1).copy()
    with np.errstate(over="ignore", invalid="ignore"):
        gt = _t((gsc * gv).astype(F32), dtype)
        if opt != ADAM and wd > 0:
            gt = _t((gt + (pv * wd).astype(F32)).astype(F32), dtype)
        m = np.ones(gv.size, bool) if not skip_zeros else (gt != 0)
        if opt == ADAM:
            n1 = (s1 * b1 + ((one - b1) * gt).astype(F32)).astype(F32)
            n2 = (s2 * b2 + ((one - b2) * (gt * gt).astype(F32)).astype(F32)).astype(F32)
            upd = (k["step_size"] * (n1 / (np.sqrt(n2).astype(F32) + k["c2eps"]).astype(F32)).astype(F32)).astype(F32)
            pn = _t((pv + upd).astype(F32), dtype)
            if wd > 0:
                pn = (pn * k["decay"]).astype(F32)
            s2 = np.where(m, n2, s2)
        elif opt == MOMENTUM:
            n1 = gt if step == 1 else (s1 * b1 + gt).astype(F32)
            pn = (pv + (-(lr * n1).astype(F32))).astype(F32)
        elif opt == LION:
            t = (s1 * b1 + ((one - b1) * gt).astype(F32)).astype(F32)
            pn = (pv - (lr * _sgn(t)).astype(F32)).astype(F32)
            n1 = (s1 * b2 + ((one - b2) * gt).astype(F32)).astype(F32)
        elif opt == RMSPROP:
            n1 = (s1 * b1 + (((one - b1) * gt).astype(F32) * gt).astype(F32)).astype(F32)
            pn = (pv - ((lr * gt).astype(F32) / (np.sqrt(n1).astype(F32) + eps).astype(F32)).astype(F32)).astype(F32)
        else:
            n1 = (s1 + (gt * gt).astype(F32)).astype(F32)
            pn = (pv - ((lr * gt).astype(F32) / (np.sqrt(n1).astype(F32) + eps).astype(F32)).astype(F32)).astype(F32)
        s1 = np.where(m, n1, s1)
        pn = np.where(m, pn, pv)
    return cast_out(pn, dtype), s1, s2
