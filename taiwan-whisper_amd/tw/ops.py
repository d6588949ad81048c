"""Typed host wrappers over libtw_hip.so.

Every wrapper validates dtypes, devices, alignment and — before any launch — that each
operand's storage really holds every element the kernel will touch, so a wrong shape
raises here instead of faulting the GPU.  All launches go on torch's current HIP stream.
"""
from __future__ import annotations

import torch

from ._native import call
from .profiling import KernelTimer

F32, BF16, F16 = 0, 1, 2
GEMM_BIAS, GEMM_ROUND, GEMM_GELU, GEMM_RES, GEMM_ACCUM, GEMM_AUX_OUT, GEMM_DGELU = 1, 2, 4, 8, 16, 32, 64
GEMM_CLAMP16 = 128     # fp16 GEMMs: clamp after the residual add (HF fp16 encoder layer, modeling_whisper.py:409-411)
HALF = (torch.bfloat16, torch.float16)
GEMM_TILE128, GEMM_TILE256, GEMM_TILE256x128, GEMM_TILE256PP = 256, 512, 1024, 2048   # forced tiles (A/B benchmarking)
GEMM_NOSPLIT = 16384   # no split-K for dW-shaped calls (A/B benchmarking)


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float16:
        return F16
    raise TypeError(f"tw: unsupported dtype {t.dtype}")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


def _need(t: torch.Tensor, n_elems: int, what: str):
    """Storage behind t (from t's first element) must hold n_elems elements."""
    if t is None:
        raise ValueError(f"tw: {what} is required")
    if not t.is_cuda:
        raise ValueError(f"tw: {what} must be a device tensor")
    st = t.untyped_storage()
    avail = (st.data_ptr() + st.nbytes() - t.data_ptr()) // t.element_size()
    if n_elems > avail:
        raise ValueError(f"tw: {what} needs {n_elems} elements past its start, storage has {avail}")


def gemm(A, B, C, M, N, K, *, lda, ldb, ldc, a_trans=False, b_trans=False, alpha=1.0, bias=None, res=None,
         ldr=0, res_mod=0, aux=None, ldaux=0, flags=0, batch=1, sA=0, sB=0, sC=0, sR=0, sAux=0, algo_N=None,
         batch_inner=1, sA_in=0, sB_in=0, sC_in=0):
    """C[b] = epi(alpha * A[b] @ B[b]^T); A [M][K] (a_trans: [K][M]); B [N][K] (b_trans: [K][N]).
    bf16 operands -> tw_gemm_bf16 (autocast rounding points); fp16 operands -> tw_gemm_f16 (the fp16 model and
    fp16-autocast training: every 16-bit tensor fp16); fp32 operands -> tw_gemm_f32 (the fp32 path: every
    operand and epilogue tensor fp32, nothing rounded)."""
    if M <= 0 or N <= 0:
        return C
    if A.dtype == torch.float32 or B.dtype == torch.float32:
        return gemm_f32(A, B, C, M, N, K, lda=lda, ldb=ldb, ldc=ldc, a_trans=a_trans, b_trans=b_trans, alpha=alpha,
                        bias=bias, res=res, ldr=ldr, res_mod=res_mod, aux=aux, ldaux=ldaux, flags=flags, batch=batch,
                        sA=sA, sB=sB, sC=sC, sR=sR, sAux=sAux, algo_N=algo_N, batch_inner=batch_inner, sA_in=sA_in,
                        sB_in=sB_in, sC_in=sC_in)
    assert batch_inner == 1, "tw.gemm: two-level batches are an fp32-path feature"
    h = A.dtype
    assert h in HALF and B.dtype == h, "tw.gemm: A and B must be both bf16, both fp16 (or both fp32)"
    assert C.dtype in (h, torch.float32), "tw.gemm: C is the operand dtype or fp32"
    _need(A, (batch - 1) * sA + ((K - 1) * lda + M if a_trans else (M - 1) * lda + K), "gemm A")
    _need(B, (batch - 1) * sB + ((K - 1) * ldb + N if b_trans else (N - 1) * ldb + K), "gemm B")
    _need(C, (batch - 1) * sC + (M - 1) * ldc + N, "gemm C")
    if bias is not None:
        assert bias.dtype == h
        _need(bias, N, "gemm bias")
        flags |= GEMM_BIAS
    if res is not None:
        assert res.dtype in (h, torch.float32)
        rows = res_mod if res_mod > 0 else M
        _need(res, (batch - 1) * sR + (rows - 1) * ldr + N, "gemm residual")
        flags |= GEMM_RES
    if aux is not None:
        assert aux.dtype == h
        _need(aux, (batch - 1) * sAux + (M - 1) * ldaux + N, "gemm aux")
    fam = "gemm_" + ("t" if a_trans else "n") + ("t" if b_trans else "n")
    flops = 2.0 * M * (N if algo_N is None else algo_N) * K * batch
    eh, ec = A.element_size(), C.element_size()
    nbytes = batch * (eh * (M * K + N * K) + ec * M * N + (res.element_size() * M * N if res is not None else 0)
                      + (eh * M * N if aux is not None else 0))
    KernelTimer.wrap(fam, flops, lambda: call(
        "tw_gemm_f16" if h == torch.float16 else "tw_gemm_bf16", A.data_ptr(), lda, int(a_trans), B.data_ptr(), ldb, int(b_trans), C.data_ptr(), ldc, _dt(C),
        M, N, K, batch, sA, sB, sC, float(alpha), _ptr(bias), _ptr(res), ldr, sR,
        _dt(res) if res is not None else F32, res_mod, _ptr(aux), ldaux, sAux, flags, _stream()), nbytes)
    return C


def gemv(x, W, C, *, ln_w=None, ln_b=None, eps=1e-5, bias=None, res=None, aux=None, flags=0, kv=None):
    """tw_gemv_bf16 / tw_gemv_f16: C[m] = epi(A[m] . W^T) for M <= 8 rows, A = x or LayerNorm(x) (ln_w / ln_b given):
    the batch-1 decode step's LN + Linear pairs in one launch (include/tw_hip.h).  kv = (cache, sb, ld, col0,
    t_dev, t_max): columns >= col0 also go to cache row *t_dev (the fused KV append)."""
    M, K = x.shape
    N = W.shape[0]
    h = x.dtype
    assert h in HALF and W.dtype == h and M <= 8 and W.shape[1] == K
    assert x.stride(1) == 1 and W.is_contiguous()
    _need(C, (M - 1) * C.stride(0) + N, "gemv C")
    if ln_w is not None:
        assert ln_w.dtype == torch.float32 and ln_b.dtype == torch.float32 and ln_w.numel() == K == ln_b.numel()
    if bias is not None:
        assert bias.dtype == h and bias.numel() >= N
        flags |= GEMM_BIAS
    if res is not None:
        _need(res, (M - 1) * res.stride(0) + N, "gemv residual")
        flags |= GEMM_RES
    if aux is not None:
        assert aux.dtype == h
        _need(aux, (M - 1) * aux.stride(0) + N, "gemv aux")
    kc, ksb, kld, kcol, kt = None, 0, 0, 0, None
    if kv is not None:
        kc, ksb, kld, kcol, kt, tmax = kv
        assert kc.dtype == C.dtype and kt.dtype == torch.int32 and 0 <= kcol < N
        _need(kc, (M - 1) * ksb + (tmax - 1) * kld + (N - kcol), "gemv kv cache")
    KernelTimer.wrap("gemv", 2.0 * M * N * K, lambda: call(
        "tw_gemv_f16" if h == torch.float16 else "tw_gemv_bf16", x.data_ptr(), x.stride(0), _ptr(ln_w), _ptr(ln_b), float(eps), W.data_ptr(), K, C.data_ptr(),
        C.stride(0), _dt(C), M, N, K, _ptr(bias), _ptr(res), res.stride(0) if res is not None else 0,
        _dt(res) if res is not None else F32, _ptr(aux), aux.stride(0) if aux is not None else 0, flags,
        _ptr(kc), ksb, kld, kcol, _ptr(kt), _stream()))
    return C


def layernorm_fwd(x, w, b, y, mean=None, rstd=None, eps=1e-5):
    D = x.shape[-1]
    rows = x.numel() // D
    assert x.is_contiguous() and y.is_contiguous() and y.numel() == x.numel()
    assert w.dtype == torch.float32 and b.dtype == torch.float32 and w.numel() == D and b.numel() == D
    if mean is not None:
        _need(mean, rows, "ln mean"); _need(rstd, rows, "ln rstd")
    call("tw_layernorm_fwd", x.data_ptr(), _dt(x), w.data_ptr(), b.data_ptr(), y.data_ptr(), _dt(y),
         _ptr(mean), _ptr(rstd), rows, D, float(eps), _stream())
    return y


def add_layernorm_fwd(x, r, x_out, w, b, y, mean=None, rstd=None, eps=1e-5):
    """x_out = x + r (fp32 or bf16 residual stream + the preceding Linear's bf16 output), y = bf16 LN(x_out); fp16
    autocast: fp32 stream, r and y fp16 (tw_add_layernorm_fwd_f16)."""
    D = x.shape[-1]
    rows = x.numel() // D
    h = r.dtype
    assert h in HALF and y.dtype == h and x_out.dtype == x.dtype
    assert x.dtype in ((torch.float32, torch.bfloat16) if h == torch.bfloat16 else (torch.float32,))
    for t in (x, r, x_out, y):
        assert t.is_contiguous() and t.numel() == x.numel() and t.is_cuda
    assert w.dtype == torch.float32 and b.dtype == torch.float32 and w.numel() == D and b.numel() == D
    if mean is not None:
        _need(mean, rows, "ln mean"); _need(rstd, rows, "ln rstd")
    call("tw_add_layernorm_fwd_f16" if h == torch.float16 else "tw_add_layernorm_fwd", x.data_ptr(), _dt(x),
         r.data_ptr(), x_out.data_ptr(), w.data_ptr(), b.data_ptr(),
         y.data_ptr(), _ptr(mean), _ptr(rstd), rows, D, float(eps), _stream())
    return y


def layernorm_bwd(x, w, mean, rstd, dy, dx, dw, db, dx_accum=True, workspace=None, g16=None):
    """dx (+)= LayerNorm backward; g16 (optional, bf16 / fp16, dx's shape): the 16-bit rounding of the final dx."""
    D = x.shape[-1]
    rows = x.numel() // D
    assert dx.dtype == torch.float32 and dx.numel() == x.numel() and dy.numel() == x.numel()
    nblk = min(1024, (rows + 3) // 4)
    if workspace is None or workspace.numel() < nblk * 2 * D:
        workspace = torch.empty(nblk * 2 * D, dtype=torch.float32, device=x.device)
    if g16 is None:
        call("tw_layernorm_bwd", x.data_ptr(), _dt(x), w.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dy.data_ptr(),
             _dt(dy), dx.data_ptr(), int(dx_accum), _ptr(dw), _ptr(db), rows, D, workspace.data_ptr(),
             workspace.numel(), _stream())
        return dx
    assert g16.dtype in HALF and g16.is_contiguous() and g16.numel() == dx.numel() and dx.is_contiguous()
    call("tw_layernorm_bwd_ex", x.data_ptr(), _dt(x), w.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dy.data_ptr(),
         _dt(dy), dx.data_ptr(), int(dx_accum), _ptr(dw), _ptr(db), rows, D, workspace.data_ptr(), workspace.numel(),
         g16.data_ptr(), _dt(g16), _stream())
    return dx


def attn_fwd(q, ldq, k, ldk, v, ldv, o, ldo, lse, B, H, Tq, Tk, causal, scale):
    if q.dtype == torch.float32:
        return attn_fwd_f32(q, ldq, k, ldk, v, ldv, o, ldo, lse, B, H, Tq, Tk, causal, scale)
    hd = 64
    for t, ld, T, nm in ((q, ldq, Tq, "q"), (k, ldk, Tk, "k"), (v, ldv, Tk, "v"), (o, ldo, Tq, "o")):
        assert t.dtype == q.dtype and t.dtype in HALF, nm
        _need(t, (B * T - 1) * ld + H * hd, f"attn {nm}")
    if lse is not None:
        _need(lse, B * H * Tq, "attn lse")
    call("tw_attn_fwd_f16" if q.dtype == torch.float16 else "tw_attn_fwd", q.data_ptr(), ldq, k.data_ptr(), ldk, v.data_ptr(), ldv, o.data_ptr(), ldo, _ptr(lse),
         B, H, Tq, Tk, hd, int(causal), float(scale), _stream())
    return o


def attn_bwd(q, ldq, k, ldk, v, ldv, o, ldo, do, lddo, lse, dq, lddq, dk, lddk, dv, lddv, B, H, Tq, Tk, causal,
             scale, workspace=None):
    if q.dtype == torch.float32:
        return attn_bwd_f32(q, ldq, k, ldk, v, ldv, o, ldo, do, lddo, lse, dq, lddq, dk, lddk, dv, lddv, B, H, Tq, Tk,
                            causal, scale)
    hd = 64
    for t, ld, T, nm in ((q, ldq, Tq, "q"), (k, ldk, Tk, "k"), (v, ldv, Tk, "v"), (o, ldo, Tq, "o"),
                         (do, lddo, Tq, "do"), (dq, lddq, Tq, "dq"), (dk, lddk, Tk, "dk"), (dv, lddv, Tk, "dv")):
        assert t.dtype == q.dtype and t.dtype in HALF, nm
        _need(t, (B * T - 1) * ld + H * hd, f"attn_bwd {nm}")
    _need(lse, B * H * Tq, "attn lse")
    if workspace is None or workspace.numel() < B * H * Tq:
        workspace = torch.empty(B * H * Tq, dtype=torch.float32, device=q.device)
    call("tw_attn_bwd_f16" if q.dtype == torch.float16 else "tw_attn_bwd", q.data_ptr(), ldq, k.data_ptr(), ldk, v.data_ptr(), ldv, o.data_ptr(), ldo, do.data_ptr(),
         lddo, lse.data_ptr(), dq.data_ptr(), lddq, dk.data_ptr(), lddk, dv.data_ptr(), lddv, B, H, Tq, Tk, hd,
         int(causal), float(scale), workspace.data_ptr(), _stream())


def kl_ce(s_logits, t_logits, labels, V, n_valid, T=2.0, ce_w=0.8, kl_w=1.0, grad_scale=1.0, dlogits=None,
          row_out=None, out3=None):
    rows, ld = s_logits.shape
    assert t_logits.shape == s_logits.shape and s_logits.dtype == t_logits.dtype
    assert s_logits.dtype in (torch.bfloat16, torch.float16, torch.float32)   # fp16: eval CE of an fp16 model
    assert labels.dtype == torch.int64 and labels.numel() == rows and n_valid.dtype == torch.int32
    if row_out is None:
        row_out = torch.empty(rows * 2, dtype=torch.float32, device=s_logits.device)
    if out3 is None:
        out3 = torch.empty(3, dtype=torch.float32, device=s_logits.device)
    if dlogits is not None:     # may be s_logits itself (in place)
        assert dlogits.shape == s_logits.shape and dlogits.dtype == s_logits.dtype
        assert dlogits.data_ptr() != t_logits.data_ptr(), "kl_ce: dlogits may alias the student logits, not the teacher's"
    call("tw_kl_ce", s_logits.data_ptr(), t_logits.data_ptr(), ld, _dt(s_logits), labels.data_ptr(), rows, V, float(T),
         float(ce_w), float(kl_w), n_valid.data_ptr(), float(grad_scale), row_out.data_ptr(), out3.data_ptr(),
         _ptr(dlogits), _stream())
    return out3, row_out


def logmel(wav, basis, mel_start, mel_w, mel_out, conv_in=None, workspace=None):
    """wav [B, n] fp32 -> mel_out [B, 80, n // 160] (+ conv_in [B, n // 160 + 2, 80] bf16).  n = 480 000 is the
    30 s path (tw_logmel); any other n > 200 is the long-form path (tw_logmel_len)."""
    B, n = wav.shape
    nfr = n // 160
    assert wav.dtype == torch.float32 and wav.is_contiguous() and n > 200
    assert mel_out.shape == (B, 80, nfr) and mel_out.dtype == torch.float32 and mel_out.is_contiguous()
    if conv_in is not None:
        assert conv_in.shape == (B, nfr + 2, 80) and conv_in.dtype == torch.bfloat16 and conv_in.is_contiguous()
    if workspace is None:
        workspace = torch.empty(B, dtype=torch.int32, device=wav.device)
    if n == 480000:
        call("tw_logmel", wav.data_ptr(), B, basis.data_ptr(), mel_start.data_ptr(), mel_w.data_ptr(),
             mel_out.data_ptr(), _ptr(conv_in), workspace.data_ptr(), _stream())
    else:
        call("tw_logmel_len", wav.data_ptr(), B, n, basis.data_ptr(), mel_start.data_ptr(), mel_w.data_ptr(),
             mel_out.data_ptr(), _ptr(conv_in), workspace.data_ptr(), _stream())
    return mel_out


def mel_to_conv_input(mel, xt):
    B, nmel, T = mel.shape
    assert xt.shape == (B, T + 2, nmel) and mel.is_contiguous() and mel.dtype == torch.float32
    if xt.dtype == torch.float32:
        call("tw_mel_to_conv_input_f32", mel.data_ptr(), xt.data_ptr(), B, nmel, T, _stream())
        return xt
    assert xt.dtype in HALF
    call("tw_mel_to_conv_input_f16" if xt.dtype == torch.float16 else "tw_mel_to_conv_input", mel.data_ptr(),
         xt.data_ptr(), B, nmel, T, _stream())
    return xt


def embed_fwd(ids, tok, pos, out, T, pos_offset=0):
    rows = ids.numel()
    D = tok.shape[1]
    assert ids.dtype == torch.int64 and out.shape[-1] == D and out.numel() == rows * D
    assert pos.shape[0] >= T + pos_offset
    call("tw_embed_fwd", ids.data_ptr(), tok.data_ptr(), _dt(tok), pos.data_ptr(), _dt(pos), out.data_ptr(),
         _dt(out), rows, T, pos_offset, D, _stream())
    return out


def embed_bwd(ids, dh, dE, padding_idx=-1):
    """dE[id] += sum of dh rows with that id (position order); ids == padding_idx skipped (nn.Embedding)."""
    rows = ids.numel()
    D = dE.shape[1]
    assert dh.dtype == torch.float32 and dE.dtype == torch.float32 and dh.numel() == rows * D
    assert ids.dtype == torch.int64 and ids.is_contiguous()
    call("tw_embed_bwd", ids.data_ptr(), dh.data_ptr(), dE.data_ptr(), rows, D, int(padding_idx), _stream())


def transpose_bf16(src, dst):
    """dst [cols][rows] = src [rows][cols]^T (16-bit words: bf16 or fp16, both row-major, dst contiguous)."""
    rows, cols = src.shape
    assert src.dtype in HALF and dst.dtype == src.dtype and src.stride(1) == 1
    assert dst.is_contiguous() and tuple(dst.shape) == (cols, rows) and src.is_cuda and dst.is_cuda
    _need(src, (rows - 1) * src.stride(0) + cols, "transpose src")
    call("tw_transpose_bf16", src.data_ptr(), src.stride(0), rows, cols, dst.data_ptr(), rows, _stream())
    return dst


def cast_bf16(src, dst):
    """fp32 -> the 16-bit dtype of dst (bf16: tw_cast_f32_bf16, fp16: tw_cast_f32_f16), RNE: autocast's weight cast
    and the rounding of a gradient entering a 16-bit GEMM operand."""
    assert src.dtype == torch.float32 and dst.dtype in HALF and src.numel() <= dst.numel()
    assert src.is_contiguous() and dst.is_contiguous()
    call("tw_cast_f32_f16" if dst.dtype == torch.float16 else "tw_cast_f32_bf16", src.data_ptr(), dst.data_ptr(),
         src.numel(), _stream())
    return dst


_WS = {}


def workspace(n, device, key="ws"):
    """Grow-only per-device scratch buffer (stream-ordered reuse)."""
    k = (key, str(device))
    t = _WS.get(k)
    if t is None or t.numel() < n:
        t = torch.empty(max(n, 1 << 16), dtype=torch.float32, device=device)
        _WS[k] = t
    return t


def colsum(x, ldx, rows, cols, out, accum=True, round_bf16=True):
    """out (+)= [round](column sums of x); round_bf16: False / True (bf16) / 2 (fp16)."""
    _need(x, (rows - 1) * ldx + cols, "colsum x")
    assert out.dtype == torch.float32 and out.numel() >= cols
    n = (rows + 63) // 64 * cols           # one fp32 partial row per 64-row chunk (tw_colsum)
    ws = workspace(n, x.device, "colsum")
    call("tw_colsum", x.data_ptr(), _dt(x), ldx, rows, cols, out.data_ptr(), int(accum), int(round_bf16),
         ws.data_ptr(), ws.numel(), _stream())


def l2norm(x, out, workspace):
    assert x.dtype == torch.float32 and x.is_contiguous() and workspace.numel() >= 1024
    call("tw_l2norm", x.data_ptr(), x.numel(), out.data_ptr(), workspace.data_ptr(), _stream())
    return out


def adamw(p, g, m, v, p_bf16, lr, b1, b2, eps, wd, step, norm=None, max_norm=0.0, inv_scale=1.0):
    """Clip + AdamW (+ the 16-bit weight copy, bf16 or fp16 by p_bf16's dtype).  inv_scale != 1: g / norm are the
    loss-scaled gradient and its norm (fp16 autocast's GradScaler; 1 / scale, a power of two)."""
    n = p.numel()
    assert g.numel() == n and m.numel() == n and v.numel() == n
    if p_bf16 is not None:
        assert p_bf16.numel() >= n and p_bf16.dtype in HALF
    if inv_scale == 1.0 and (p_bf16 is None or p_bf16.dtype == torch.bfloat16):
        call("tw_adamw", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), _ptr(p_bf16), n, float(lr), float(b1),
             float(b2), float(eps), float(wd), int(step), _ptr(norm), float(max_norm), _stream())
        return
    call("tw_adamw_ex", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), _ptr(p_bf16),
         F16 if p_bf16 is not None and p_bf16.dtype == torch.float16 else BF16, n, float(lr), float(b1), float(b2),
         float(eps), float(wd), int(step), _ptr(norm), float(max_norm), float(inv_scale), _stream())


def im2col3(src, src_rows, dst, B, T_out, stride, C):
    _need(src, (B - 1) * src_rows * C + ((T_out - 1) * stride + 3) * C, "im2col src")
    _need(dst, B * T_out * 3 * C, "im2col dst")
    assert src.dtype == dst.dtype
    fn = "tw_im2col3_f32" if src.dtype == torch.float32 else "tw_im2col3"
    call(fn, src.data_ptr(), src_rows, dst.data_ptr(), B, T_out, stride, C, _stream())


def col2im_s2(dA, dX, B, T_in, T_out, C):
    assert dA.dtype == torch.float32 and dX.dtype == torch.float32
    _need(dA, B * T_out * 3 * C, "col2im dA"); _need(dX, B * T_in * C, "col2im dX")
    call("tw_col2im_s2", dA.data_ptr(), dX.data_ptr(), B, T_in, T_out, C, _stream())


def shift_tokens_right(labels, out, pad, start):
    B, T = labels.shape
    assert labels.dtype == torch.int64 and out.shape == labels.shape and labels.is_contiguous()
    call("tw_shift_tokens_right", labels.data_ptr(), out.data_ptr(), B, T, pad, start, _stream())
    return out


def count_valid(labels, out):
    assert labels.dtype == torch.int64 and out.dtype == torch.int32
    call("tw_count_valid", labels.data_ptr(), labels.numel(), out.data_ptr(), _stream())
    return out


def gelu_bwd(g, pre, out):
    assert g.numel() == pre.numel() == out.numel()
    if pre.dtype == torch.float32:
        assert g.dtype == torch.float32 and out.dtype == torch.float32
        call("tw_gelu_bwd_f32", g.data_ptr(), pre.data_ptr(), out.data_ptr(), g.numel(), _stream())
        return out
    assert pre.dtype in HALF and out.dtype == pre.dtype
    call("tw_gelu_bwd_f16" if pre.dtype == torch.float16 else "tw_gelu_bwd", g.data_ptr(), _dt(g), pre.data_ptr(),
         out.data_ptr(), g.numel(), _stream())
    return out


# ----------------------------------------------------------------------------- greedy decode (A12)
def decode_attn(q, sqb, k, ldk, skb, v, ldv, svb, o, sob, B, H, Tk, scale, tk_dev=None, tk_max=None, hsk=None,
                hsv=None):
    """One query row per (b, h) over the first Tk (+ *tk_dev) cached key rows (include/tw_hip.h).
    With tk_dev the host cannot know Tk: tk_max bounds the rows checked for extent.  hsk / hsv: head strides of
    K / V (tw_decode_attn_hs; default 64, heads side by side in a row); skb = svb = 0 shares one clip's K/V."""
    hd = 64
    for t, nm in ((q, "q"), (k, "k"), (v, "v"), (o, "o")):
        assert t.dtype == q.dtype and t.dtype in (torch.bfloat16, torch.float16, torch.float32), nm
    rows = Tk if tk_dev is None else tk_max
    hk, hv = (hd if hsk is None else int(hsk)), (hd if hsv is None else int(hsv))
    _need(q, (B - 1) * sqb + H * hd, "decode q")
    _need(k, (B - 1) * skb + (rows - 1) * ldk + (H - 1) * hk + hd, "decode k")
    _need(v, (B - 1) * svb + (rows - 1) * ldv + (H - 1) * hv + hd, "decode v")
    _need(o, (B - 1) * sob + H * hd, "decode o")
    if tk_dev is not None:
        assert tk_dev.dtype == torch.int32 and tk_max is not None
    # algorithmic bytes (KernelTimer family "decode_attn_cross" / "decode_attn_self"): every K and V
    # element of the rows attended once (self: the host does not know *tk_dev; tk_max bounds it)
    work = 2 * B * rows * H * hd * q.element_size()
    if hsk is None and hsv is None:
        fn = lambda: call("tw_decode_attn", q.data_ptr(), sqb, k.data_ptr(), ldk, skb, v.data_ptr(), ldv, svb,
                          o.data_ptr(), sob, B, H, Tk, _ptr(tk_dev), hd, float(scale), _dt(q), _stream())
    else:
        fn = lambda: call("tw_decode_attn_hs", q.data_ptr(), sqb, k.data_ptr(), ldk, skb, hk, v.data_ptr(), ldv, svb,
                          hv, o.data_ptr(), sob, B, H, Tk, _ptr(tk_dev), hd, float(scale), _dt(q), _stream())
    KernelTimer.wrap("decode_attn_self" if tk_dev is not None else "decode_attn_cross", work, fn)
    return o


def token_bitmask(ids, V, device):
    """V-bit uint32 mask (as int32 storage) with the given token ids set."""
    words = torch.zeros((V + 31) // 32, dtype=torch.int64)
    for i in ids:
        i = int(i)
        if 0 <= i < V:
            words[i >> 5] |= 1 << (i & 31)
    words = torch.where(words >= 2 ** 31, words - 2 ** 32, words)
    return words.to(torch.int32).to(device)


def greedy_select(logits, ld, B, V, suppress_bits, begin_bits, apply_begin, eos, done, ids, col, next_ids,
                  t_dev=None, begin_col=-1):
    assert logits.dtype in (torch.bfloat16, torch.float16, torch.float32) and ids.dtype == torch.int64
    assert next_ids.dtype == torch.int64 and done.dtype == torch.uint8
    _need(logits, (B - 1) * ld + V, "greedy logits")
    _need(ids, (B - 1) * ids.stride(0) + (ids.shape[1] if t_dev is not None else col + 1), "greedy ids")
    _need(done, B, "greedy done"); _need(next_ids, B, "greedy next")
    for m, nm in ((suppress_bits, "suppress"), (begin_bits, "begin")):
        if m is not None:
            _need(m, (V + 31) // 32, f"greedy {nm} mask")
    call("tw_greedy_select", logits.data_ptr(), ld, _dt(logits), B, V, _ptr(suppress_bits), _ptr(begin_bits), int(apply_begin),
         int(eos), done.data_ptr(), ids.data_ptr(), ids.stride(0), col, next_ids.data_ptr(), _ptr(t_dev),
         int(begin_col), _stream())


def greedy_select_ts(logits, ld, B, V, suppress_bits, begin_bits, eos, done, ids, col, next_ids, last_ts,
                     begin_col, ts_begin=50364, no_ts=50363, max_initial=-1, t_dev=None):
    assert logits.dtype in (torch.bfloat16, torch.float16, torch.float32) and ids.dtype == torch.int64
    assert next_ids.dtype == torch.int64 and done.dtype == torch.uint8 and last_ts.dtype == torch.int32
    _need(logits, (B - 1) * ld + V, "greedy logits")
    _need(ids, (B - 1) * ids.stride(0) + (ids.shape[1] if t_dev is not None else col + 1), "greedy ids")
    _need(done, B, "greedy done"); _need(next_ids, B, "greedy next"); _need(last_ts, B, "greedy last_ts")
    for m, nm in ((suppress_bits, "suppress"), (begin_bits, "begin")):
        if m is not None:
            _need(m, (V + 31) // 32, f"greedy {nm} mask")
    call("tw_greedy_select_ts", logits.data_ptr(), ld, _dt(logits), B, V, _ptr(suppress_bits), _ptr(begin_bits), int(eos),
         done.data_ptr(), ids.data_ptr(), ids.stride(0), col, next_ids.data_ptr(), _ptr(t_dev), int(begin_col),
         int(ts_begin), int(no_ts), int(max_initial if max_initial is not None else -1), last_ts.data_ptr(),
         _stream())


def select_sample(logits, ld, B, V, suppress_bits, begin_bits, apply_begin, eos, done, ids, col, next_ids, ctl,
                  sum_logp, t_dev=None, begin_col=-1):
    """greedy_select + temperature sampling (ctl: int32[3B], per row bits(1/T), seed lo, hi; 1/T = 0 -> argmax)
    + running log-prob of the chosen token (sum_logp: float32[B])."""
    assert ctl.dtype == torch.int32 and ctl.numel() >= 3 * B and sum_logp.dtype == torch.float32
    _need(sum_logp, B, "select sum_logp")
    assert logits.dtype in (torch.bfloat16, torch.float16, torch.float32) and ids.dtype == torch.int64
    assert next_ids.dtype == torch.int64 and done.dtype == torch.uint8
    _need(logits, (B - 1) * ld + V, "select logits")
    _need(ids, (B - 1) * ids.stride(0) + (ids.shape[1] if t_dev is not None else col + 1), "select ids")
    _need(done, B, "select done"); _need(next_ids, B, "select next")
    call("tw_select_sample", logits.data_ptr(), ld, _dt(logits), B, V, _ptr(suppress_bits), _ptr(begin_bits), int(apply_begin),
         int(eos), done.data_ptr(), ids.data_ptr(), ids.stride(0), col, next_ids.data_ptr(), _ptr(t_dev),
         int(begin_col), ctl.data_ptr(), sum_logp.data_ptr(), _stream())


def select_sample_ts(logits, ld, B, V, suppress_bits, begin_bits, eos, done, ids, col, next_ids, last_ts, begin_col,
                     ctl, sum_logp, ts_begin=50364, no_ts=50363, max_initial=-1, t_dev=None):
    assert ctl.dtype == torch.int32 and ctl.numel() >= 3 * B and sum_logp.dtype == torch.float32
    _need(sum_logp, B, "select sum_logp")
    assert logits.dtype in (torch.bfloat16, torch.float16, torch.float32) and ids.dtype == torch.int64
    assert next_ids.dtype == torch.int64 and done.dtype == torch.uint8 and last_ts.dtype == torch.int32
    _need(logits, (B - 1) * ld + V, "select logits")
    _need(ids, (B - 1) * ids.stride(0) + (ids.shape[1] if t_dev is not None else col + 1), "select ids")
    _need(done, B, "select done"); _need(next_ids, B, "select next"); _need(last_ts, B, "select last_ts")
    call("tw_select_sample_ts", logits.data_ptr(), ld, _dt(logits), B, V, _ptr(suppress_bits), _ptr(begin_bits), int(eos),
         done.data_ptr(), ids.data_ptr(), ids.stride(0), col, next_ids.data_ptr(), _ptr(t_dev), int(begin_col),
         int(ts_begin), int(no_ts), int(max_initial if max_initial is not None else -1), last_ts.data_ptr(),
         ctl.data_ptr(), sum_logp.data_ptr(), _stream())


def token_logprob(logits, ld, B, V, token, out):
    """out[b] = log_softmax(logits[b, :V])[token] (float32)."""
    assert logits.dtype in (torch.bfloat16, torch.float16, torch.float32) and out.dtype == torch.float32
    _need(logits, (B - 1) * ld + V, "token_logprob logits"); _need(out, B, "token_logprob out")
    call("tw_token_logprob", logits.data_ptr(), ld, _dt(logits), B, V, int(token), out.data_ptr(), _stream())
    return out


def sample_ctl(temperature, seed, out=None):
    """Device control words of select_sample[_ts], one per row: [bits(1/T) (0 = greedy), seed lo, seed hi] x B.
    temperature / seed: scalars (one row) or equal-length sequences (a batch of independent attempts)."""
    import struct
    temps = list(temperature) if isinstance(temperature, (list, tuple)) else [temperature]
    seeds = list(seed) if isinstance(seed, (list, tuple)) else [seed] * len(temps)
    assert len(seeds) == len(temps)
    vals = []
    for t, sd in zip(temps, seeds):
        inv = 0.0 if not t or t <= 0 else 1.0 / float(t)
        bits = struct.unpack("<i", struct.pack("<f", inv))[0]
        sd = int(sd) & ((1 << 64) - 1)
        lo, hi = sd & 0xFFFFFFFF, sd >> 32
        vals += [bits, lo - (1 << 32) if lo >= 1 << 31 else lo, hi - (1 << 32) if hi >= 1 << 31 else hi]
    vals = torch.tensor(vals, dtype=torch.int32)
    if out is None:
        return vals
    assert out.numel() >= vals.numel()
    out[:vals.numel()].copy_(vals)
    return out


def embed_step(ids, tok, pos, out, t_dev, max_pos):
    B = ids.numel()
    D = tok.shape[1]
    assert ids.dtype == torch.int64 and t_dev.dtype == torch.int32 and out.numel() == B * D
    assert pos.shape[0] >= max_pos
    call("tw_embed_step", ids.data_ptr(), tok.data_ptr(), _dt(tok), pos.data_ptr(), _dt(pos), out.data_ptr(),
         _dt(out), B, D, t_dev.data_ptr(), _stream())
    return out


def kv_append(src, ld_src, cache, ld_row, sb, B, n, t_dev, max_rows):
    assert src.dtype == cache.dtype and src.dtype in (torch.bfloat16, torch.float16, torch.float32) and t_dev.dtype == torch.int32
    _need(src, (B - 1) * ld_src + n, "kv_append src")
    _need(cache, (B - 1) * sb + (max_rows - 1) * ld_row + n, "kv_append cache")
    call("tw_kv_append", src.data_ptr(), ld_src, cache.data_ptr(), ld_row, sb, B, n, _dt(src), t_dev.data_ptr(),
         _stream())


def kv_head_major(src, ld, dst, B, Tk, H):
    """Row-interleaved cross K/V [B*Tk][ld] -> head-major K [B][H][Tk][64] then V (include/tw_hip.h)."""
    assert src.dtype == dst.dtype and src.dtype in (torch.bfloat16, torch.float16, torch.float32)
    _need(src, (B * Tk - 1) * ld + 2 * 64 * H, "kv_head_major src")
    _need(dst, 2 * B * H * Tk * 64, "kv_head_major dst")
    call("tw_kv_head_major", src.data_ptr(), ld, dst.data_ptr(), B, Tk, H, _dt(src), _stream())


def step_advance(t_dev, by=1):
    assert t_dev.dtype == torch.int32 and t_dev.is_cuda
    call("tw_step_advance", t_dev.data_ptr(), int(by), _stream())


# ----------------------------------------------------------------------------- fp32 arithmetic path
def gemm_f32(A, B, C, M, N, K, *, lda, ldb, ldc, a_trans=False, b_trans=False, alpha=1.0, bias=None, res=None,
             ldr=0, res_mod=0, aux=None, ldaux=0, flags=0, batch=1, sA=0, sB=0, sC=0, sR=0, sAux=0, algo_N=None,
             batch_inner=1, sA_in=0, sB_in=0, sC_in=0):
    """tw_gemm_f32: every tensor fp32; batch entry bz = bo * batch_inner + bi at offsets bo*s? + bi*s?_in."""
    if M <= 0 or N <= 0:
        return C
    for t, nm in ((A, "A"), (B, "B"), (C, "C"), (bias, "bias"), (res, "res"), (aux, "aux")):
        assert t is None or t.dtype == torch.float32, f"tw.gemm_f32: {nm} must be fp32"
    assert batch % batch_inner == 0
    nb = batch // batch_inner
    _need(A, (nb - 1) * sA + (batch_inner - 1) * sA_in + ((K - 1) * lda + M if a_trans else (M - 1) * lda + K),
          "gemm_f32 A")
    _need(B, (nb - 1) * sB + (batch_inner - 1) * sB_in + ((K - 1) * ldb + N if b_trans else (N - 1) * ldb + K),
          "gemm_f32 B")
    _need(C, (nb - 1) * sC + (batch_inner - 1) * sC_in + (M - 1) * ldc + N, "gemm_f32 C")
    flags &= ~GEMM_ROUND
    if bias is not None:
        _need(bias, N, "gemm_f32 bias")
        flags |= GEMM_BIAS
    if res is not None:
        rows = res_mod if res_mod > 0 else M
        _need(res, (nb - 1) * sR + (rows - 1) * ldr + N, "gemm_f32 residual")
        flags |= GEMM_RES
    if aux is not None:
        _need(aux, (nb - 1) * sAux + (M - 1) * ldaux + N, "gemm_f32 aux")
    fam = "gemm32_" + ("t" if a_trans else "n") + ("t" if b_trans else "n")
    flops = 2.0 * M * (N if algo_N is None else algo_N) * K * batch
    eh, ec = A.element_size(), C.element_size()
    nbytes = batch * (eh * (M * K + N * K) + ec * M * N + (res.element_size() * M * N if res is not None else 0)
                      + (eh * M * N if aux is not None else 0))
    KernelTimer.wrap(fam, flops, lambda: call(
        "tw_gemm_f32", A.data_ptr(), lda, int(a_trans), B.data_ptr(), ldb, int(b_trans), C.data_ptr(), ldc, M, N, K,
        batch, sA, sB, sC, batch_inner, sA_in, sB_in, sC_in, float(alpha), _ptr(bias), _ptr(res), ldr, sR, res_mod,
        _ptr(aux), ldaux, sAux, flags, _stream()), nbytes)
    return C


def _attn_ws(Tq, Tk, bufs, device, B, H):
    """score workspace: as many (b, h) pairs per pass as fit in 512 MiB (at least one)."""
    per = Tq * ((Tk + 3) // 4 * 4) * bufs
    n = max(per, min(B * H * per, (512 << 20) // 4))
    return workspace(n, device, "attn_f32"), n


def attn_fwd_f32(q, ldq, k, ldk, v, ldv, o, ldo, lse, B, H, Tq, Tk, causal, scale):
    hd = 64
    for t, ld, T, nm in ((q, ldq, Tq, "q"), (k, ldk, Tk, "k"), (v, ldv, Tk, "v"), (o, ldo, Tq, "o")):
        assert t.dtype == torch.float32, nm
        _need(t, (B * T - 1) * ld + H * hd, f"attn_f32 {nm}")
    if lse is not None:
        _need(lse, B * H * Tq, "attn_f32 lse")
    ws, n = _attn_ws(Tq, Tk, 1, q.device, B, H)
    call("tw_attn_fwd_f32", q.data_ptr(), ldq, k.data_ptr(), ldk, v.data_ptr(), ldv, o.data_ptr(), ldo, _ptr(lse),
         B, H, Tq, Tk, hd, int(causal), float(scale), ws.data_ptr(), n, _stream())
    return o


def attn_bwd_f32(q, ldq, k, ldk, v, ldv, o, ldo, do, lddo, lse, dq, lddq, dk, lddk, dv, lddv, B, H, Tq, Tk, causal,
                 scale):
    hd = 64
    for t, ld, T, nm in ((q, ldq, Tq, "q"), (k, ldk, Tk, "k"), (v, ldv, Tk, "v"), (o, ldo, Tq, "o"),
                         (do, lddo, Tq, "do"), (dq, lddq, Tq, "dq"), (dk, lddk, Tk, "dk"), (dv, lddv, Tk, "dv")):
        assert t.dtype == torch.float32, nm
        _need(t, (B * T - 1) * ld + H * hd, f"attn_bwd_f32 {nm}")
    _need(lse, B * H * Tq, "attn_bwd_f32 lse")
    ws, n = _attn_ws(Tq, Tk, 2, q.device, B, H)
    call("tw_attn_bwd_f32", q.data_ptr(), ldq, k.data_ptr(), ldk, v.data_ptr(), ldv, o.data_ptr(), ldo, do.data_ptr(),
         lddo, lse.data_ptr(), dq.data_ptr(), lddq, dk.data_ptr(), lddk, dv.data_ptr(), lddv, B, H, Tq, Tk, hd,
         int(causal), float(scale), ws.data_ptr(), n, _stream())
