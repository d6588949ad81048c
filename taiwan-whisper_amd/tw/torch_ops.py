"""The HIP kernels as PyTorch operators: `torch.ops.tw.*` (the C-ABI "wrapped by TORCH_LIBRARY(tw, ...)"
with autograd for the trainable pieces).

Each op is a `torch.library.custom_op` over the same C-ABI entry points the engine calls (tw/ops.py -> libtw_hip.so),
so it runs the identical kernel with identical arguments: a layer composed from these ops is bit-identical to the
engine's own ctypes path (tests/test_torch_ops_gpu.py).  Every op has a fake (meta) implementation, so it can be traced
(torch.compile / torch.export / FakeTensor), and the trainable ones register their backward (register_autograd), so
`loss.backward()` runs the HIP backward kernels.  Device: cuda (the HIP build); there is no CPU kernel -- a CPU tensor
raises, as the engine does.

Arithmetic (autocast rounding points), reference call sites:
  tw::linear            y = round16(x W^T + b)                              nn.Linear under autocast (HF modeling_whisper.py)
  tw::linear_gelu       pre = round16(x W^T + b), y = round16(gelu(pre))    fc1 + exact-erf GELU (HF :325, activations.py:70)
  tw::linear_residual   out = res + round16(x W^T + b)  (res fp32 / 16-bit) out_proj / fc2 + the residual add (HF :392-413)
  tw::layer_norm        y = round16(LN(x)) (+ mean, rstd)                    nn.LayerNorm (fp32 statistics)
  tw::attention         o = softmax(q k^T * scale [causal]) v (+ lse)        SDPA (HF attention interface :337-350)
  tw::kl_ce             (loss, ce, kl), dloss/ds                              run_distillation.py:1507-1516, 1539-1549
  tw::log_mel           [B, n] fp32 -> [B, 80, n // 160] fp32                  WhisperFeatureExtractor (HF :135-170)
Backward products use the same kernels as tw.modeling.Backward (bf16 dX / dW / bias sums, rounded as autocast rounds
them); the 16-bit forward ops accept bf16 and fp16 (fp16: forward only, as the engine's fp16 model).
"""
from __future__ import annotations

import functools
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import ops as F

HALF = (torch.bfloat16, torch.float16)


def _rows(x: Tensor) -> Tuple[int, int]:
    assert x.dim() == 2 and x.stride(1) == 1, "tw ops: 2-D operand with unit column stride"
    return x.shape[0], x.shape[1]


def _gemm_fwd(x, w, b, out, flags, res=None, aux=None):
    M, K = _rows(x)
    N = w.shape[0]
    assert w.shape[1] == K and w.is_contiguous() and w.dtype == x.dtype
    F.gemm(x, w, out, M, N, K, lda=x.stride(0), ldb=K, ldc=out.stride(0), bias=b, res=res,
           ldr=res.stride(0) if res is not None else 0, aux=aux, ldaux=aux.stride(0) if aux is not None else 0,
           flags=flags)
    return out


def _lin_bwd(g, x, w, need_b):
    """dX = round(g W), dW = round(g^T x), db = round(colsum g) (bf16, as tw.modeling.Backward)."""
    if g.dtype != torch.bfloat16:
        raise NotImplementedError("tw ops: backward is a bf16 (autocast) path; the fp16 model is forward-only")
    g = g.contiguous()
    M, N = g.shape
    K = x.shape[1]
    dx = torch.empty(M, K, dtype=torch.bfloat16, device=g.device)
    F.gemm(g, w, dx, M, K, N, lda=N, ldb=K, ldc=K, b_trans=True, flags=F.GEMM_ROUND)
    dw = torch.empty(N, K, dtype=torch.float32, device=g.device)
    F.gemm(g, x, dw, N, K, M, lda=N, ldb=x.stride(0), ldc=K, a_trans=True, b_trans=True, flags=F.GEMM_ROUND)
    db = None
    if need_b:
        db = torch.empty(N, dtype=torch.float32, device=g.device)
        F.colsum(g, N, M, N, db, accum=False, round_bf16=True)
        db = db.to(w.dtype)
    return dx, dw.to(w.dtype), db


# ------------------------------------------------------------------------------------------------ linear
@torch.library.custom_op("tw::linear", mutates_args=(), device_types="cuda")
def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor]) -> Tensor:
    out = torch.empty(x.shape[0], weight.shape[0], dtype=x.dtype, device=x.device)
    return _gemm_fwd(x, weight, bias, out, F.GEMM_ROUND)


@linear.register_fake
def _(x, weight, bias):
    return x.new_empty(x.shape[0], weight.shape[0])


def _linear_setup(ctx, inputs, output):
    x, w, b = inputs
    ctx.save_for_backward(x, w)
    ctx.has_b = b is not None


def _linear_bwd(ctx, g):
    x, w = ctx.saved_tensors
    dx, dw, db = _lin_bwd(g, x, w, ctx.has_b)
    return dx.to(x.dtype), dw, db


linear.register_autograd(_linear_bwd, setup_context=_linear_setup)


# ------------------------------------------------------------------------------------------------ linear + GELU
@torch.library.custom_op("tw::linear_gelu", mutates_args=(), device_types="cuda")
def linear_gelu(x: Tensor, weight: Tensor, bias: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    out = torch.empty(x.shape[0], weight.shape[0], dtype=x.dtype, device=x.device)
    pre = torch.empty_like(out)
    _gemm_fwd(x, weight, bias, out, F.GEMM_ROUND | F.GEMM_GELU | F.GEMM_AUX_OUT, aux=pre)
    return out, pre


@linear_gelu.register_fake
def _(x, weight, bias):
    o = x.new_empty(x.shape[0], weight.shape[0])
    return o, torch.empty_like(o)


def _linear_gelu_setup(ctx, inputs, output):
    x, w, b = inputs
    ctx.save_for_backward(x, w, output[1])
    ctx.has_b = b is not None
    ctx.mark_non_differentiable(output[1])


def _linear_gelu_bwd(ctx, g, _gpre):
    x, w, pre = ctx.saved_tensors
    if g.dtype != torch.bfloat16 or pre.dtype != torch.bfloat16:
        raise NotImplementedError("tw ops: backward is a bf16 (autocast) path; the fp16 model is forward-only")
    dpre = torch.empty_like(pre)
    F.gelu_bwd(g.contiguous(), pre, dpre)             # round16(g * gelu'(pre)): the DGELU epilogue's arithmetic
    dx, dw, db = _lin_bwd(dpre, x, w, ctx.has_b)
    return dx.to(x.dtype), dw, db


linear_gelu.register_autograd(_linear_gelu_bwd, setup_context=_linear_gelu_setup)


# ------------------------------------------------------------------------------------------------ linear + residual
@torch.library.custom_op("tw::linear_residual", mutates_args=(), device_types="cuda")
def linear_residual(x: Tensor, weight: Tensor, bias: Optional[Tensor], res: Tensor) -> Tensor:
    assert res.dtype in (x.dtype, torch.float32) and res.shape == (x.shape[0], weight.shape[0])
    out = torch.empty(res.shape, dtype=res.dtype, device=x.device)
    return _gemm_fwd(x, weight, bias, out, F.GEMM_ROUND, res=res.contiguous())


@linear_residual.register_fake
def _(x, weight, bias, res):
    return res.new_empty(res.shape)


def _linear_res_setup(ctx, inputs, output):
    x, w, b, _ = inputs
    ctx.save_for_backward(x, w)
    ctx.has_b = b is not None


def _linear_res_bwd(ctx, g):
    x, w = ctx.saved_tensors
    g16 = g.to(torch.bfloat16) if g.dtype == torch.float32 else g   # the grad entering the bf16 Linear output
    dx, dw, db = _lin_bwd(g16, x, w, ctx.has_b)
    return dx.to(x.dtype), dw, db, g


linear_residual.register_autograd(_linear_res_bwd, setup_context=_linear_res_setup)


# ------------------------------------------------------------------------------------------------ LayerNorm
@torch.library.custom_op("tw::layer_norm", mutates_args=(), device_types="cuda")
def layer_norm(x: Tensor, weight: Tensor, bias: Tensor, eps: float) -> Tuple[Tensor, Tensor, Tensor]:
    """y in the 16-bit compute dtype (bf16 for an fp32 / bf16 input, fp16 for fp16); weight / bias fp32."""
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=torch.float16 if x.dtype == torch.float16 else torch.bfloat16, device=x.device)
    mean = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    F.layernorm_fwd(x, weight, bias, y, mean, rstd, eps=eps)
    return y, mean, rstd


@layer_norm.register_fake
def _(x, weight, bias, eps):
    y = torch.empty(x.shape, dtype=torch.float16 if x.dtype == torch.float16 else torch.bfloat16, device=x.device)
    m = x.new_empty(x.shape[0], dtype=torch.float32)
    return y, m, torch.empty_like(m)


def _ln_setup(ctx, inputs, output):
    x, w, b, eps = inputs
    ctx.save_for_backward(x.contiguous(), w, output[1], output[2])
    ctx.mark_non_differentiable(output[1], output[2])


def _ln_bwd(ctx, dy, _dm, _dr):
    x, w, mean, rstd = ctx.saved_tensors
    dx = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    dw = torch.zeros_like(w)
    db = torch.zeros_like(w)
    F.layernorm_bwd(x, w, mean, rstd, dy.contiguous(), dx, dw, db, dx_accum=False)
    return dx.to(x.dtype), dw, db, None


layer_norm.register_autograd(_ln_bwd, setup_context=_ln_setup)


# ------------------------------------------------------------------------------------------------ attention
def _heads(t: Tensor):
    """[B, T, H*64] view whose rows may be strided (a column slice of a fused projection) -> (ld, H)."""
    assert t.dim() == 3 and t.stride(2) == 1 and t.shape[2] % 64 == 0
    B, T, C = t.shape
    assert B == 1 or t.stride(0) == T * t.stride(1), "tw::attention: rows of a batch must be contiguous"
    return t.stride(1), C // 64


@torch.library.custom_op("tw::attention", mutates_args=(), device_types="cuda")
def attention(q: Tensor, k: Tensor, v: Tensor, causal: bool, scale: float) -> Tuple[Tensor, Tensor]:
    """q [B, Tq, H*64], k / v [B, Tk, H*64] (16-bit) -> o [B, Tq, H*64], lse [B*H*Tq] fp32."""
    ldq, H = _heads(q)
    ldk, _ = _heads(k)
    ldv, _ = _heads(v)
    B, Tq, C = q.shape
    Tk = k.shape[1]
    o = torch.empty(B, Tq, C, dtype=q.dtype, device=q.device)
    lse = torch.empty(B * H * Tq, dtype=torch.float32, device=q.device)
    F.attn_fwd(q, ldq, k, ldk, v, ldv, o, C, lse, B, H, Tq, Tk, causal, scale)
    return o, lse


@attention.register_fake
def _(q, k, v, causal, scale):
    B, Tq, C = q.shape
    return q.new_empty(B, Tq, C), q.new_empty(B * (C // 64) * Tq, dtype=torch.float32)


def _attn_setup(ctx, inputs, output):
    q, k, v, causal, scale = inputs
    ctx.save_for_backward(q, k, v, output[0], output[1])
    ctx.causal, ctx.scale = causal, scale
    ctx.mark_non_differentiable(output[1])


def _attn_bwd(ctx, do, _dlse):
    q, k, v, o, lse = ctx.saved_tensors
    if q.dtype != torch.bfloat16:
        raise NotImplementedError("tw::attention backward is a bf16 (autocast) path")
    ldq, H = _heads(q)
    ldk, _ = _heads(k)
    ldv, _ = _heads(v)
    B, Tq, C = q.shape
    Tk = k.shape[1]
    do = do.contiguous()
    dq, dk, dv = torch.empty_like(o), torch.empty(B, Tk, C, dtype=q.dtype, device=q.device), \
        torch.empty(B, Tk, C, dtype=q.dtype, device=q.device)
    F.attn_bwd(q, ldq, k, ldk, v, ldv, o, C, do, C, lse, dq, C, dk, C, dv, C, B, H, Tq, Tk, ctx.causal, ctx.scale)
    return dq, dk, dv, None, None


attention.register_autograd(_attn_bwd, setup_context=_attn_setup)


# ------------------------------------------------------------------------------------------------ KL + CE
@torch.library.custom_op("tw::kl_ce", mutates_args=(), device_types="cuda")
def kl_ce(s_logits: Tensor, t_logits: Tensor, labels: Tensor, vocab_size: int, temperature: float, ce_weight: float,
          kl_weight: float) -> Tuple[Tensor, Tensor]:
    """-> (out3 = [loss, ce, kl] fp32, dloss/ds_logits in the logits' dtype).  The fused kernel produces the gradient
    of the combined loss (out3[0]) in the same pass; autograd scales it by that output's incoming gradient."""
    lab = labels.reshape(-1).contiguous()
    nv = torch.zeros(1, dtype=torch.int32, device=s_logits.device)
    F.count_valid(lab, nv)
    dl = torch.empty_like(s_logits)
    out3, _ = F.kl_ce(s_logits, t_logits, lab, vocab_size, nv, T=temperature, ce_w=ce_weight, kl_w=kl_weight,
                      dlogits=dl)
    return out3, dl


@kl_ce.register_fake
def _(s_logits, t_logits, labels, vocab_size, temperature, ce_weight, kl_weight):
    return s_logits.new_empty(3, dtype=torch.float32), torch.empty_like(s_logits)


def _klce_setup(ctx, inputs, output):
    ctx.save_for_backward(output[1])
    ctx.mark_non_differentiable(output[1])


def _klce_bwd(ctx, g3, _gdl):
    (dl,) = ctx.saved_tensors
    # d out3[0] only (the loss run_distillation.py backpropagates, :1549, :1665); ce / kl are reported values
    return (dl * g3[0].to(dl.dtype)), None, None, None, None, None, None


kl_ce.register_autograd(_klce_bwd, setup_context=_klce_setup)


# ------------------------------------------------------------------------------------------------ log-mel
@functools.lru_cache(maxsize=None)
def _mel_tables(device: str):
    from .feature_extraction import mel_tables
    return mel_tables(device)


@torch.library.custom_op("tw::log_mel", mutates_args=(), device_types="cuda")
def log_mel(wav: Tensor) -> Tensor:
    """[B, n] fp32 waveform (16 kHz; n = 480 000 for a 30 s window, any n > 200 for long-form) -> [B, 80, n // 160]."""
    wav = wav.contiguous()
    B, n = wav.shape
    basis, start, w = _mel_tables(str(wav.device))
    mel = torch.empty(B, 80, n // 160, dtype=torch.float32, device=wav.device)
    F.logmel(wav, basis, start, w, mel)
    return mel


@log_mel.register_fake
def _(wav):
    return wav.new_empty(wav.shape[0], 80, wav.shape[1] // 160)


OPS = ("linear", "linear_gelu", "linear_residual", "layer_norm", "attention", "kl_ce", "log_mel")
