"""fp16 distillation (the reference's --dtype float16: run_distillation.py:815-817 mixed_precision="fp16", the teacher
loaded in fp16 (:1009-1018), accelerate's GradScaler around the backward) on the GPU.

Kernels: the fp16 instantiations added for training -- tw_gemm_f16 with transposed operands (dX, dW, split-K dW),
tw_attn_bwd_f16, tw_gelu_bwd_f16, tw_cast_f32_f16, tw_colsum with fp16 rounding, tw_adamw_ex (fp16 weight copy,
GradScaler.unscale_ folded in) -- each against an fp64 / torch reference on the same fp16 inputs, with the
tolerance stated in the test (one fp16 ulp = 2^-11 relative where an output is rounded to fp16).

Step: tests/golden/cfg_c{1,2,3,3b10}.npz rows "f16|..." (tests/golden/make_golden.py gen_cfg_f16): HF Transformers under
torch.autocast(float16) with an fp16 teacher and a default GradScaler (scale 2^16), unscale_ -> clip_grad_norm_ ->
scaler.step -> scaler.update.  Bars as tests/test_configs_gpu.py with the fixture's own fp16 noise: every tensor
within 2 x dist(HF fp16, HF fp32) of HF fp16 and 2.5 x of HF fp32 (floors 1e-2 per-tensor norm, 2e-3 total norm),
loss / CE / KL within 1e-3 of both, the fc1 update's sign on >= 99.5 % of elements, and the loss scale after the
step equal to HF's."""
import math

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from tw import _native
    _native.lib()


def h(x):
    return x.to(torch.float16)


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-30))


# ----------------------------------------------------------------------------- kernels
@pytest.mark.parametrize("a_t,b_t", [(0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(200, 136, 72), (257, 520, 1280), (4096, 768, 768)])
def test_gemm_f16_transposed_layouts(a_t, b_t, M, N, K):
    """fp16 operands, fp32 output: only the fp32 accumulation order differs from fp64 (1e-5 of the largest)."""
    from tw import ops
    if (a_t and M % 8) or (b_t and N % 8):
        pytest.skip("MN-major operands need 8-aligned extents")
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K)
    A, Bm = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    ref = h(A).double() @ h(Bm).double().T
    Ad = h(A.T.contiguous() if a_t else A).to(DEV)
    Bd = h(Bm.T.contiguous() if b_t else Bm).to(DEV)
    C = torch.zeros(M, N, dtype=torch.float32, device=DEV)
    ops.gemm(Ad, Bd, C, M, N, K, lda=M if a_t else K, ldb=N if b_t else K, ldc=N, a_trans=bool(a_t),
             b_trans=bool(b_t))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < 1e-5


def test_gemm_f16_dx_dgelu_epilogue():
    """dX = fp16(fp16(dY W) * gelu'(pre)) on the transposed-B kernel (the MLP backward of fp16 autocast) vs the fp64
    value rounded at the same two points: the fp32 accumulation may flip the inner rounding by one ulp, so two fp16
    ulps (2^-9 relative) plus one ulp of the fp16 subnormal range (2^-24) where the product is tiny."""
    from tw import ops
    g = torch.Generator().manual_seed(5)
    M, N, K = 1024, 768, 3072
    dy, w, pre = h(torch.randn(M, N, generator=g)), h(torch.randn(N, K, generator=g) * 0.05), h(torch.randn(M, K, generator=g))
    out = torch.empty(M, K, dtype=torch.float16, device=DEV)
    ops.gemm(dy.to(DEV), w.to(DEV), out, M, K, N, lda=N, ldb=K, ldc=K, b_trans=True, aux=pre.to(DEV), ldaux=K,
             flags=ops.GEMM_ROUND | ops.GEMM_DGELU)
    torch.cuda.synchronize()
    x = pre.double()
    gp = 0.5 * (1 + torch.erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)
    ref = h(h(dy.double() @ w.double()).double() * gp).double()
    d = (out.cpu().double() - ref).abs()
    # + the fp32 accumulation term where dY W cancels: 1e-6 of sum |dY||W| (K = 768 fp32 adds), times gelu'
    cancel = 1e-6 * (dy.double().abs() @ w.double().abs()) * gp.abs()
    bad = d > 2 ** -9 * ref.abs() + 2 ** -24 + cancel
    assert not bool(bad.any()), (int(bad.sum()), float(d.max()))


@pytest.mark.parametrize("M,N,K,flags", [(28608, 5120, 1280, "gelu_aux"), (28608, 1280, 5120, "res32"),
                                          (28608, 51904, 1280, "store"), (1000, 2560, 1280, "store")])
def test_gemm_f16_ragged_full_tiles_plus_edges_bit_identical(M, N, K, flags):
    """fp16 grids ragged in M or N (the fp16 teacher decoder's M = 64 x 447, the LM head's N = 51 904): the whole
    256x256 tiles on the persistent kernel, the edge strips on the 128x128 kernel -- bit-identical to the 128x128
    kernel alone (same K order per output)."""
    from tw import ops
    g = torch.Generator().manual_seed(M + N + K)
    A = h(torch.randn(M, K, generator=g)).to(DEV)
    W = h(torch.randn(N, K, generator=g) * 0.03).to(DEV)
    bias = h(torch.randn(N, generator=g) * 0.1).to(DEV)
    outs = []
    for forced in (0, ops.GEMM_TILE128):
        kw = {}
        if flags == "gelu_aux":
            C = torch.empty(M, N, dtype=torch.float16, device=DEV)
            kw = dict(aux=torch.empty(M, N, dtype=torch.float16, device=DEV), ldaux=N,
                      flags=ops.GEMM_ROUND | ops.GEMM_GELU | ops.GEMM_AUX_OUT | forced)
        elif flags == "res32":
            C = torch.linspace(-3, 3, M * N, device=DEV).view(M, N).contiguous()
            kw = dict(res=C, ldr=N, flags=ops.GEMM_ROUND | forced)
        else:
            C = torch.empty(M, N, dtype=torch.float16, device=DEV)
            kw = dict(flags=ops.GEMM_ROUND | forced)
        ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bias, **kw)
        torch.cuda.synchronize()
        outs.append((C.clone(), kw.get("aux")))
    assert torch.equal(outs[0][0], outs[1][0])
    if flags == "gelu_aux":
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("D", [768, 1280])
def test_add_layernorm_f16_matches_residual_epilogue(D):
    """fp16 autocast's deferred residual update (fp32 stream + fp16 Linear output r, then the LayerNorm with fp16
    output: tw_add_layernorm_fwd_f16) == the fp16 GEMM's fp32 residual epilogue followed by tw_layernorm_fwd, bit for
    bit, in place and into a separate stream buffer."""
    from tw import ops
    g = torch.Generator().manual_seed(D + 7)
    rows, K = 1000, 256
    x0 = (torch.randn(rows, D, generator=g) * 3).to(DEV)
    A, W = h(torch.randn(rows, K, generator=g)).to(DEV), h(torch.randn(D, K, generator=g) * 0.1).to(DEV)
    bias = h(torch.randn(D, generator=g)).to(DEV)
    w, b = torch.randn(D, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)
    xa = x0.clone()
    ops.gemm(A, W, xa, rows, D, K, lda=K, ldb=K, ldc=D, bias=bias, res=xa, ldr=D, flags=ops.GEMM_ROUND)
    ya = torch.empty(rows, D, dtype=torch.float16, device=DEV)
    ma, ra = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
    ops.layernorm_fwd(xa, w, b, ya, ma, ra)
    r = torch.empty(rows, D, dtype=torch.float16, device=DEV)
    ops.gemm(A, W, r, rows, D, K, lda=K, ldb=K, ldc=D, bias=bias, flags=ops.GEMM_ROUND)
    for inplace in (True, False):
        xb = x0.clone()
        xo = xb if inplace else torch.empty_like(xb)
        yb = torch.empty_like(ya)
        mb, rb = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
        ops.add_layernorm_fwd(xb, r, xo, w, b, yb, mb, rb)
        torch.cuda.synchronize()
        assert torch.equal(xo, xa) and torch.equal(yb, ya) and torch.equal(mb, ma) and torch.equal(rb, ra)


@pytest.mark.parametrize("N,K,M", [(768, 768, 14304), (264, 136, 4096), (1280, 1280, 1000)])
def test_gemm_f16_splitk_weight_grad(N, K, M):
    """dW += fp16(dY^T X) through the split-K path vs the unsplit kernel: one fp16 ulp of the product plus the fp32
    regrouping term (2e-5 of the largest product), and both within 1e-3 of fp64."""
    from tw import ops
    g = torch.Generator().manual_seed(N + K + M)
    dy, x = torch.randn(M, N, generator=g) * 0.1, torch.randn(M, K, generator=g)
    dyd, xd = h(dy).to(DEV), h(x).to(DEV)
    base = torch.randn(N, K, generator=g)
    ref = h((h(dy).double().T @ h(x).double()).float()).double() + base.double()
    outs = []
    for f in (0, ops.GEMM_NOSPLIT):
        dw = base.clone().to(DEV)
        ops.gemm(dyd, xd, dw, N, K, M, lda=N, ldb=K, ldc=K, a_trans=True, b_trans=True,
                 flags=ops.GEMM_ROUND | ops.GEMM_ACCUM | f)
        torch.cuda.synchronize()
        outs.append(dw.cpu())
    prod = torch.maximum((outs[0] - base).abs(), (outs[1] - base).abs())
    tol = prod * 2 ** -10 + 2e-5 * float(prod.max())
    d = (outs[0] - outs[1]).abs()
    assert not bool((d > tol).any()), float(d.max())
    assert rel_err(outs[0], ref) < 1e-3 and rel_err(outs[1], ref) < 1e-3


@pytest.mark.parametrize("B,H,Tq,Tk,causal", [(2, 3, 200, 200, True), (1, 2, 447, 1500, False), (1, 2, 5, 70, False)])
def test_attention_f16_fwd_bwd(B, H, Tq, Tk, causal):
    """fp16 flash attention forward + backward vs fp64 autograd on the same fp16 inputs (P and dS are rounded to fp16
    for their MFMAs: 1e-2 of the largest gradient, 4x tighter than the bf16 bar)."""
    from tw import ops
    g = torch.Generator().manual_seed(Tq * 3 + Tk)
    d = H * 64
    qq_ = h(torch.randn(B * Tq, d, generator=g))
    kv = h(torch.randn(B * Tk, 2 * d, generator=g))
    qd, kvd = qq_.to(DEV), kv.to(DEV)
    o = torch.empty(B * Tq, d, dtype=torch.float16, device=DEV)
    lse = torch.empty(B * H * Tq, device=DEV)
    ops.attn_fwd(qd, d, kvd, 2 * d, kvd[:, d:], 2 * d, o, d, lse, B, H, Tq, Tk, causal, 0.125)
    sh = lambda t, T: t.double().view(B, T, H, 64).transpose(1, 2)
    q, k, v = (sh(t, T).requires_grad_(True) for t, T in ((qq_, Tq), (kv[:, :d], Tk), (kv[:, d:], Tk)))
    s = (q @ k.transpose(-1, -2)) * 0.125
    if causal:
        s = s.masked_fill(torch.ones(Tq, Tk, dtype=torch.bool).triu(1 + Tk - Tq), float("-inf"))
    out = torch.softmax(s, -1) @ v
    ref = out.detach().transpose(1, 2).reshape(B * Tq, d)
    assert rel_err(o.float(), ref) < 3e-3
    do = h(torch.randn(B, H, Tq, 64, generator=g))
    out.backward(do.double())
    dod = do.transpose(1, 2).reshape(B * Tq, d).contiguous().to(DEV)
    dq = torch.empty(B * Tq, d, dtype=torch.float16, device=DEV)
    dkv = torch.empty(B * Tk, 2 * d, dtype=torch.float16, device=DEV)
    ops.attn_bwd(qd, d, kvd, 2 * d, kvd[:, d:], 2 * d, o, d, dod, d, lse, dq, d, dkv, 2 * d, dkv[:, d:], 2 * d,
                 B, H, Tq, Tk, causal, 0.125)
    torch.cuda.synchronize()
    back = lambda t, T: t.transpose(1, 2).reshape(B * T, d)
    for got, want, nm in ((dq, back(q.grad, Tq), "dq"), (dkv[:, :d], back(k.grad, Tk), "dk"),
                          (dkv[:, d:], back(v.grad, Tk), "dv")):
        e = rel_err(got.float(), want)
        assert e < 1e-2, (nm, e)


def test_f16_helpers_cast_colsum_gelu_bwd():
    from tw import ops
    g = torch.Generator().manual_seed(11)
    x = torch.randn(70001, generator=g) * 3
    dst = torch.empty(70001, dtype=torch.float16, device=DEV)
    ops.cast_bf16(x.to(DEV), dst)
    assert torch.equal(dst.cpu(), x.half())           # RNE, as torch's .half()
    rows, cols = 4097, 768
    a = h(torch.randn(rows, cols, generator=g))
    out = torch.ones(cols, device=DEV)
    ops.colsum(a.to(DEV), cols, rows, cols, out, accum=True, round_bf16=2)
    ref = a.double().sum(0).float().half().float() + 1.0
    assert (out.cpu() - ref).abs().max() <= 2 ** -10 * ref.abs().max()
    gg, pre = torch.randn(50000, generator=g), h(torch.randn(50000, generator=g) * 2)
    o = torch.empty(50000, dtype=torch.float16, device=DEV)
    ops.gelu_bwd(gg.to(DEV), pre.to(DEV), o)
    xx = pre.double()
    gp = 0.5 * (1 + torch.erf(xx / math.sqrt(2))) + xx * torch.exp(-0.5 * xx * xx) / math.sqrt(2 * math.pi)
    ref = (gg.half().double() * gp).half().double()
    d = (o.cpu().double() - ref).abs()     # one rounding after an fp32 product: one fp16 ulp (subnormals: 2^-24)
    assert not bool((d > 2 ** -10 * ref.abs() + 2 ** -24).any()), float(d.max())


def test_adamw_ex_unscale_is_exact():
    """tw_adamw_ex on the loss-scaled gradient with inv_scale = 2^-16 == tw_adamw on the unscaled gradient and its
    norm (bit for bit: scaling by a power of two is exact), and the fp16 copy of the weights is their RNE cast."""
    from tw import ops
    g = torch.Generator().manual_seed(3)
    n = 100003
    p0 = torch.randn(n, generator=g).to(DEV)
    gr = (torch.randn(n, generator=g) * 1e-3).to(DEV)
    scale = 65536.0
    gs = gr * scale
    m0, v0 = (torch.rand(n, generator=g) * 1e-4).to(DEV), (torch.rand(n, generator=g) * 1e-6).to(DEV)
    norm = torch.tensor([float(gr.double().norm())], device=DEV, dtype=torch.float32)
    norm_s = norm * scale
    pa, ma, va = p0.clone(), m0.clone(), v0.clone()
    pb, mb, vb = p0.clone(), m0.clone(), v0.clone()
    w16 = torch.empty(n, dtype=torch.float16, device=DEV)
    ops.adamw(pa, gr, ma, va, None, 1e-4, 0.9, 0.999, 1e-8, 0.01, 3, norm, 0.5)
    ops.adamw(pb, gs, mb, vb, w16, 1e-4, 0.9, 0.999, 1e-8, 0.01, 3, norm_s, 0.5, inv_scale=1.0 / scale)
    torch.cuda.synchronize()
    assert torch.equal(pa, pb) and torch.equal(ma, mb) and torch.equal(va, vb)
    assert torch.equal(w16, pb.half())


# ----------------------------------------------------------------------------- the step vs HF fp16 autocast
def _build(name):
    import oracle.fixture_inputs as mg
    from oracle.weights import CONFIGS, make_weights
    from tw.config import WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    from tw.student import student_from_teacher
    g = load_golden("cfg_" + name)
    if "f16|loss" not in g:
        pytest.skip(f"cfg_{name}.npz has no fp16 rows")
    c = mg.CFG_CASES[name]
    dev = torch.device("cuda", 0)
    tcfg = CONFIGS[c["teacher"]]
    wt = make_weights(tcfg, c["t_seed"], per_tensor=True, embed_std=mg.EMBED_STD)
    sd = {k: torch.from_numpy(v) for k, v in wt.items()}
    if c["student"] is None:
        t32 = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**tcfg), sd, dtype=torch.float32,
                                                              device=dev)
        s, _, _ = student_from_teacher(t32, decoder_layers=2)
        del t32
        s.set_compute("fp16")
    else:
        scfg = CONFIGS[c["student"]]
        ws = make_weights(scfg, c["s_seed"], per_tensor=True, embed_std=mg.EMBED_STD)
        s = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**scfg),
                                                            {k: torch.from_numpy(v) for k, v in ws.items()},
                                                            dtype=torch.float32, device=dev, compute="fp16")
    t = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**tcfg), sd, dtype=torch.float16, device=dev)
    assert s.compute == t.compute == "fp16" and s.store.p16.dtype == torch.float16
    feats, dec, lab = mg.cfg_case_batch(name)
    batch = dict(input_features=torch.from_numpy(feats).to(dev), decoder_input_ids=torch.from_numpy(dec).to(dev),
                 labels=torch.from_numpy(lab).to(dev))
    assert np.array_equal(g["dec"], dec) and np.array_equal(g["lab"], lab)
    return g, s, t, batch, c


def _rl2(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return float((a - b).norm() / b.norm())


def _maxrel(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return float(((a - b).abs() / b.abs().clamp_min(1e-30)).max())


def _within_noise(what, got, g, key, dist, floor=0.0, f16_out=False):
    ref, f32 = g["f16|" + key], g["f32|" + key]
    noise = dist(ref, f32)
    if f16_out:
        ref, f32 = (torch.as_tensor(x).to(torch.float16).float() for x in (ref, f32))
    d_ref, d_f32 = dist(got, ref), dist(got, f32)
    print(f"  {what}: dist(hip, HF fp16) {d_ref:.3e}  dist(hip, HF fp32) {d_f32:.3e}  ref noise {noise:.3e}")
    assert d_ref <= max(2.0 * noise, floor), (what, d_ref, noise)
    assert d_f32 <= max(2.5 * noise, floor), (what, d_f32, noise)


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c3b10"])   # c3b10: M >= 4096, the production GEMM routes
def test_fp16_distillation_step_at_baseline_dims(name):
    from tw.distill import DistillationTrainer
    from tw.modeling import to_hf
    g, s, t, batch, c = _build(name)
    tr = DistillationTrainer(s, t, learning_rate=1e-4, warmup_steps=0, freeze_encoder=c["freeze_encoder"],
                             freeze_embed_positions=c["freeze_embed_positions"])
    assert tr.scaler is not None and tr.scaler.scale == float(g["f16|scale"])
    names = [str(n) for n in g["grad_names"]]
    cap = {}
    orig = tr.optimizer_step

    def hook():
        cap["grad"] = s.grad.clone()
        cap["scale"] = tr.scaler.scale
        return orig()
    tr.optimizer_step = hook
    enc = s.encode(s.conv_input(batch["input_features"])).float().cpu()
    p0 = "model.decoder.layers.0.fc1.weight"
    before = s.state_view(p0)[::37, ::29].double().cpu()
    m = tr.train_step(batch)
    torch.cuda.synchronize()
    for k, fk in (("loss", "loss"), ("ce_loss", "ce"), ("kl_loss", "kl")):
        got = m[k].item()
        for mode in ("f16", "f32"):
            ref = float(g[f"{mode}|{fk}"])
            assert abs(got - ref) / abs(ref) < 1e-3, (k, mode, got, ref)
    B = batch["labels"].shape[0]
    _within_noise(name + " encoder output", enc.view(B, 1500, -1)[:, ::50, :], g, "enc_sub", _rl2, f16_out=True)
    grad = cap["grad"].double() / cap["scale"]        # the engine's gradient is loss-scaled until the update
    norms = []
    for n in names:
        o = s.store.offset[n]
        norms.append(to_hf(n, grad[o: o + s.store.numel(n)].view(s.store.segs[n]), s.config).norm().item())
    _within_noise(name + " per-tensor grad norms", np.array(norms), g, "grad_norms", _maxrel, floor=1e-2)
    _within_noise(name + " total grad norm", np.array([grad.norm().item()]),
                  {k: np.array([g[k]]) for k in ("f16|grad_total_norm", "f32|grad_total_norm")}, "grad_total_norm",
                  _maxrel, floor=2e-3)
    o = s.store.offset[p0]
    gsub = grad[o: o + s.store.numel(p0)].view(s.store.segs[p0])[::37, ::29].cpu()
    _within_noise(name + " dec0.fc1 grad block", gsub, g, "grad_dec0_fc1_sub", _rl2)
    upd = s.state_view(p0)[::37, ::29].double().cpu() - before
    want = torch.from_numpy(g["f16|upd_dec0_fc1_sub"]).double() - before
    agree = float((torch.sign(upd) == torch.sign(want)).double().mean())
    print(name, "update sign agreement", agree)
    assert agree >= 0.995, agree
    assert tr.step == 1 and tr.skipped_steps == 0
    assert tr.scaler.scale == float(g["f16|scale_after"])
    # the fp16 mirror the next forward reads is the fp16 cast of the updated master
    assert torch.equal(s.store.p16[: s.train_prefix], s.store.p32[: s.train_prefix].half())


def test_fp16_scaler_skips_overflowing_step():
    """A loss scale that overflows the fp16 loss gradient: the update is skipped (weights, moments, AdamW step and
    the schedule untouched) and the scale halves (GradScaler.update's backoff); the next finite step applies."""
    from tw.distill import DistillationTrainer
    g, s, t, batch, c = _build("c1")
    tr = DistillationTrainer(s, t, learning_rate=1e-4, freeze_encoder=True)
    p_before = s.store.p32.clone()
    tr.scaler.scale = 2.0 ** 70
    tr.train_step(batch)
    torch.cuda.synchronize()
    assert tr.skipped_steps == 1 and tr.step == 0 and tr.scaler.scale == 2.0 ** 69
    assert not math.isfinite(float(tr.norm.item()))
    assert torch.equal(s.store.p32, p_before) and float(tr.m_buf.abs().max()) == 0.0
    tr.scaler.scale = 65536.0
    tr.train_step(batch)
    torch.cuda.synchronize()
    assert tr.skipped_steps == 1 and tr.step == 1 and tr.scaler.growth_tracker == 1
    assert not torch.equal(s.store.p32, p_before)
