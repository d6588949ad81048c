"""The fp32 arithmetic path (mixed_precision = "no": the reference's default --dtype float32,
training/run_distillation.py:815-823) on the GPU.

Kernels: tw_gemm_f32 (exact-fp32 MFMA) and the composed SDPA (tw_attn_*_f32) against float64 torch on
the same fp32 inputs: relative error <= 1e-5 (GEMMs) / 2e-5 (attention), i.e. fp32 accumulation-order
noise only.

End to end, against HF Transformers run in fp32 (the fixtures of tests/golden/make_golden.py):
  * greedy decode (greedy.npz), timestamp decode (greedy_ts.npz: one window and 65 s long-form) and
    long-form with conditioning / thresholds (fallback.npz): token ids IDENTICAL to HF generate --
    north star "token ids bit-exact for greedy decode", no near-tie allowance;
  * the per-window average log-probs / no-speech probabilities of that long-form run: 1e-4;
  * the distillation step on the micro config (micro_step.npz) and at c1 / c2 / c3 dims (cfg_c*.npz
    f32|...): loss / CE / KL 2e-5 relative, per-tensor gradient norms 1e-3 relative, the sampled gradient
    block and the encoder output 1e-4 relative L2.
"""
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


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


# ------------------------------------------------------------------------------------------ kernels
@pytest.mark.parametrize("a_t,b_t", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(200, 136, 72), (131, 257, 447), (1500, 64, 1500), (3, 384, 128)])
def test_gemm_f32_layouts(a_t, b_t, M, N, K):
    from tw import ops
    if (a_t and M % 4) or (b_t and N % 4):
        pytest.skip("MN-major operands: lda / ldb = M / N must be a multiple of 4")
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K)
    A, Bm = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    ref = A.double() @ Bm.double().T
    lda = M if a_t else (K + 3) // 4 * 4
    ldb = N if b_t else (K + 3) // 4 * 4
    Ad = torch.zeros(K if a_t else M, lda, device=DEV)
    Bd = torch.zeros(K if b_t else N, ldb, device=DEV)
    if a_t:
        Ad[:, :M] = A.T.to(DEV)
    else:
        Ad[:, :K] = A.to(DEV)
    if b_t:
        Bd[:, :N] = Bm.T.to(DEV)
    else:
        Bd[:, :K] = Bm.to(DEV)
    C = torch.full((M, N), float("nan"), device=DEV)
    ops.gemm(Ad, Bd, C, M, N, K, lda=lda, ldb=ldb, ldc=N, a_trans=bool(a_t), b_trans=bool(b_t))
    torch.cuda.synchronize()
    assert rel(C, ref) < 1e-5


def test_gemm_f32_epilogues_and_batches():
    from tw import ops
    g = torch.Generator().manual_seed(2)
    M, N, K, R = 300, 264, 128, 100
    A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.1
    bias, res, pre = torch.randn(N, generator=g), torch.randn(R, N, generator=g), torch.randn(M, N, generator=g)
    Ad, Wd, bd = A.to(DEV), W.to(DEV), bias.to(DEV)
    y = A.double() @ W.double().T + bias.double()
    gelu = lambda x: 0.5 * x * (1 + torch.erf(x / np.sqrt(2)))
    # bias + GELU with the pre-activation stored
    C, aux = torch.empty(M, N, device=DEV), torch.empty(M, N, device=DEV)
    ops.gemm(Ad, Wd, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, aux=aux, ldaux=N,
             flags=ops.GEMM_GELU | ops.GEMM_AUX_OUT | ops.GEMM_ROUND)      # ROUND is ignored on fp32
    assert rel(aux, y) < 1e-5 and rel(C, gelu(y)) < 1e-5
    # bias + residual with res_mod (positional table), alpha, accumulate
    C2 = torch.ones(M, N, device=DEV)
    ops.gemm(Ad, Wd, C2, M, N, K, lda=K, ldb=K, ldc=N, alpha=0.5, bias=bd, res=res.to(DEV), ldr=N, res_mod=R,
             flags=ops.GEMM_ACCUM)
    want = 0.5 * (A.double() @ W.double().T) + bias.double() + res.double()[torch.arange(M) % R] + 1.0
    assert rel(C2, want) < 1e-5
    # DGELU: C = (A W^T) * gelu'(aux)
    C3 = torch.empty(M, N, device=DEV)
    ops.gemm(Ad, Wd, C3, M, N, K, lda=K, ldb=K, ldc=N, aux=pre.to(DEV), ldaux=N, flags=ops.GEMM_DGELU)
    x = pre.double()
    dg = 0.5 * (1 + torch.erf(x / np.sqrt(2))) + x * torch.exp(-0.5 * x * x) / np.sqrt(2 * np.pi)
    assert rel(C3, (A.double() @ W.double().T) * dg) < 1e-5
    # two batch levels: (b, h) blocks of 64 columns in shared rows, as the attention products use them
    B, H, T, hd = 3, 4, 70, 64
    X = torch.randn(B * T, H * hd, generator=g)
    Y = torch.randn(B * T, H * hd, generator=g)
    S = torch.empty(B, H, T, 72, device=DEV)
    ops.gemm(X.to(DEV), Y.to(DEV), S, T, T, hd, lda=H * hd, ldb=H * hd, ldc=72, batch=B * H, batch_inner=H,
             sA=T * H * hd, sB=T * H * hd, sC=H * T * 72, sA_in=hd, sB_in=hd, sC_in=T * 72)
    xr = X.double().view(B, T, H, hd).transpose(1, 2)
    yr = Y.double().view(B, T, H, hd).transpose(1, 2)
    assert rel(S[..., :T], xr @ yr.transpose(-1, -2)) < 1e-5


@pytest.mark.parametrize("B,H,Tq,Tk,causal", [(2, 3, 447, 447, True), (2, 2, 100, 1500, False), (1, 20, 7, 7, True),
                                              (3, 1, 1500, 1500, False)])
def test_attention_f32_fwd_bwd(B, H, Tq, Tk, causal):
    from tw import ops
    g = torch.Generator().manual_seed(B * 7 + Tq)
    d = H * 64
    q, k, v = (torch.randn(B * T, d, generator=g) for T in (Tq, Tk, Tk))
    do = torch.randn(B * Tq, d, generator=g)
    qq = q.double().view(B, Tq, H, 64).transpose(1, 2).requires_grad_(True)
    kk = k.double().view(B, Tk, H, 64).transpose(1, 2).requires_grad_(True)
    vv = v.double().view(B, Tk, H, 64).transpose(1, 2).requires_grad_(True)
    s = (qq @ kk.transpose(-1, -2)) * 0.125
    if causal:
        s = s.masked_fill(torch.ones(Tq, Tk, dtype=torch.bool).triu(1 + Tk - Tq), float("-inf"))
    out = torch.softmax(s, -1) @ vv
    out.backward(do.double().view(B, Tq, H, 64).transpose(1, 2))
    lse_ref = torch.logsumexp(s, -1)
    qd, kd, vd, dod = (t.to(DEV) for t in (q, k, v, do))
    o = torch.empty(B * Tq, d, device=DEV)
    lse = torch.empty(B * H * Tq, device=DEV)
    ops.attn_fwd(qd, d, kd, d, vd, d, o, d, lse, B, H, Tq, Tk, causal, 0.125)
    dq, dk, dv = torch.empty_like(qd), torch.empty_like(kd), torch.empty_like(vd)
    ops.attn_bwd(qd, d, kd, d, vd, d, o, d, dod, d, lse, dq, d, dk, d, dv, d, B, H, Tq, Tk, causal, 0.125)
    torch.cuda.synchronize()
    back = lambda t, T: t.transpose(1, 2).reshape(B * T, d)
    assert rel(o, back(out.detach(), Tq)) < 2e-5
    assert (lse.cpu().double() - lse_ref.reshape(-1)).abs().max() < 1e-4
    for got, want in ((dq, back(qq.grad, Tq)), (dk, back(kk.grad, Tk)), (dv, back(vv.grad, Tk))):
        assert rel(got, want) < 2e-5


# ------------------------------------------------------------------------------------ greedy decode
def _micro32(lin_std=0.2):
    from test_decode_gpu import _micro
    cfg, w, m, GC = _micro(lin_std=lin_std)
    m.set_compute("fp32")
    return cfg, w, m, GC


def test_fp32_greedy_bit_exact_vs_hf():
    from test_decode_gpu import _feats
    cfg, w, m, GC = _micro32()
    g = load_golden("greedy")
    m.generation_config = GC(suppress_tokens=g["suppress"].tolist(), begin_suppress_tokens=[220, 50257])
    prompt = torch.tensor([g["greedy_prompt"].tolist()] * 3)
    for use_graph in (True, False):
        gen = m.generate(_feats(), decoder_input_ids=prompt, max_length=64, use_graph=use_graph).cpu().numpy()
        np.testing.assert_array_equal(gen, g["greedy_ids"])


def test_fp32_timestamps_bit_exact_vs_hf():
    from test_decode_gpu import _feats, _ts_model
    mg, cfg, w, m = _ts_model()
    m.set_compute("fp32")
    g = load_golden("greedy_ts")
    feats = torch.from_numpy(np.stack([_feats()[0].numpy(), _feats()[1].numpy()]))
    gen = m.generate(feats, return_timestamps=True, language="zh", task="transcribe", max_new_tokens=48).cpu()
    np.testing.assert_array_equal(gen.numpy(), g["ts_short_ids"])
    lf = torch.from_numpy(mg.longform_features())
    out = m.generate(lf, attention_mask=torch.ones(1, lf.shape[-1], dtype=torch.long), return_timestamps=True,
                     language="zh", task="transcribe").cpu()
    np.testing.assert_array_equal(out.numpy(), g["ts_long_ids"])


def test_fp32_longform_fallback_conditioning_bit_exact_vs_hf():
    from test_decode_gpu import _ts_model
    mg, cfg, w, m = _ts_model()
    m.set_compute("fp32")
    g = load_golden("fallback")
    lf = torch.from_numpy(mg.longform_features())
    kw = dict(attention_mask=torch.ones(1, lf.shape[-1], dtype=torch.long), return_timestamps=True, language="zh",
              task="transcribe")
    cond = m.generate(lf, condition_on_prev_tokens=True, temperature=0.0, **kw).cpu().numpy()
    np.testing.assert_array_equal(cond, g["fb_cond_ids"])
    trace = []
    none = m.generate(lf, temperature=(0.0,), logprob_threshold=-1e9, no_speech_threshold=1.0, _trace=trace,
                      **kw).cpu().numpy()
    np.testing.assert_array_equal(none, g["fb_none_ids"])
    np.testing.assert_allclose([t["avg_logprob"] for t in trace], g["fb_avg_logprobs"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose([t["no_speech_prob"] for t in trace], g["fb_ns_probs"], rtol=1e-4, atol=1e-9)
    skip = m.generate(lf, temperature=(0.0,), logprob_threshold=1e9, no_speech_threshold=0.0, **kw).cpu().numpy()
    assert skip.shape[1] == 0 and g["fb_skipall_ids"].shape[1] == 0


# --------------------------------------------------------------------------------- training step
def _step_f32(cfg_s, ws, cfg_t, wt, feats, dec, lab, freeze_encoder, freeze_embed_positions=True, student=None):
    from tw.config import WhisperConfig
    from tw.distill import DistillationTrainer
    from tw.modeling import WhisperForConditionalGeneration
    mk = lambda c, w: WhisperForConditionalGeneration.from_state_dict(
        WhisperConfig(**c), {k: torch.from_numpy(v) for k, v in w.items()}, dtype=torch.float32, compute="fp32")
    s = student if student is not None else mk(cfg_s, ws)
    t = mk(cfg_t, wt)
    tr = DistillationTrainer(s, t, learning_rate=1e-4, warmup_steps=0, freeze_encoder=freeze_encoder,
                             freeze_embed_positions=freeze_embed_positions)
    cap = {}
    orig = tr.optimizer_step

    def hook():
        cap["grad"] = s.grad.clone()
        return orig()
    tr.optimizer_step = hook
    batch = dict(input_features=torch.as_tensor(feats).to(DEV), decoder_input_ids=torch.as_tensor(dec).to(DEV),
                 labels=torch.as_tensor(lab).to(DEV))
    m = tr.train_step(batch)
    torch.cuda.synchronize()
    return s, t, {k: v.item() for k, v in m.items()}, cap["grad"], batch


def _grad_norms(s, grad, names):
    from tw.modeling import to_hf
    out = []
    for n in names:
        o = s.store.offset[n]
        out.append(to_hf(n, grad[o: o + s.store.numel(n)].view(s.store.segs[n]), s.config).double().norm().item())
    return np.array(out)


def test_fp32_train_step_matches_hf_fp32_micro():
    from oracle.weights import CONFIGS, make_weights
    g = load_golden("micro_step")
    cfg = CONFIGS["micro"]
    s, t, m, grad, batch = _step_f32(cfg, make_weights(cfg, 1), cfg, make_weights(cfg, 2), g["feats"], g["dec"],
                                     g["lab"], True)
    for k, fk in (("loss", "loss"), ("ce_loss", "ce"), ("kl_loss", "kl_share")):
        assert abs(m[k] - float(g[fk])) / abs(float(g[fk])) < 2e-5, (k, m[k], float(g[fk]))
    names = [str(n) for n in g["grad_names"]]
    r = np.abs(_grad_norms(s, grad, names) - g["grad_norms"]) / g["grad_norms"]
    assert r.max() < 1e-3, (names[int(r.argmax())], r.max())
    assert abs(grad.double().norm().item() - float(g["grad_total_norm"])) / float(g["grad_total_norm"]) < 1e-4
    # AdamW after clip: first update on the sampled block equals HF's within fp32 noise of lr
    got = s.state_view("model.decoder.layers.0.self_attn.q_proj.weight")[::5, ::5].cpu().numpy()
    np.testing.assert_allclose(got, g["upd_dec0_q_sub"], atol=2e-6)
    out = s(input_features=batch["input_features"], decoder_input_ids=batch["decoder_input_ids"])
    lse = torch.logsumexp(out.logits.float(), -1).cpu()
    # weights moved by one update since the fixture's forward: compare the encoder (frozen) only
    enc = out.encoder_last_hidden_state.float().cpu()[:, ::50, :]
    assert rel(enc, torch.from_numpy(g["enc_sub"])) < 1e-4
    assert lse.shape == tuple(g["s_lse"].shape)


def test_fp32_train_step_matches_hf_fp32_c1():
    """c1 dims (tiny <- tiny, B 2, shared frozen encoder): the fp32 engine vs HF fp32."""
    import os, sys
    import oracle.fixture_inputs as mg
    g = load_golden("cfg_c1")
    scfg, ws, tcfg, wt = mg.cfg_case_weights("c1")
    feats, dec, lab = mg.cfg_case_batch("c1")
    c = mg.CFG_CASES["c1"]
    s, t, m, grad, batch = _step_f32(scfg, ws, tcfg, wt, feats, dec, lab, c["freeze_encoder"],
                                     c["freeze_embed_positions"])
    for k, fk in (("loss", "loss"), ("ce_loss", "ce"), ("kl_loss", "kl")):
        ref = float(g["f32|" + fk])
        assert abs(m[k] - ref) / abs(ref) < 2e-5, (k, m[k], ref)
    names = [str(n) for n in g["grad_names"]]
    r = np.abs(_grad_norms(s, grad, names) - g["f32|grad_norms"]) / g["f32|grad_norms"]
    assert r.max() < 1e-3, (names[int(r.argmax())], r.max())
    p0 = "model.decoder.layers.0.fc1.weight"
    o = s.store.offset[p0]
    gsub = grad[o: o + s.store.numel(p0)].view(s.store.segs[p0])[::37, ::29]
    assert rel(gsub, torch.from_numpy(g["f32|grad_dec0_fc1_sub"])) < 1e-4


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_fp32_train_step_matches_hf_fp32_large(name):
    """c2 (small <- large-v2, full teacher forward, the whole student trained incl. conv stem) and c3
    (distil-32-2 made by tw.student from the large-v2 teacher, shared frozen encoder, prompt quirk) at B=1
    on the fp32 path vs HF fp32."""
    import os, sys
    import oracle.fixture_inputs as mg
    from oracle.weights import CONFIGS, make_weights
    from tw.config import WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    from tw.student import student_from_teacher
    g = load_golden("cfg_" + name)
    c = mg.CFG_CASES[name]
    tcfg = CONFIGS[c["teacher"]]
    wt = make_weights(tcfg, c["t_seed"], per_tensor=True, embed_std=mg.EMBED_STD)
    feats, dec, lab = mg.cfg_case_batch(name)
    student, scfg, ws = None, None, None
    if c["student"] is None:
        t32 = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**tcfg), {k: torch.from_numpy(v) for k, v in
                                                                                      wt.items()}, dtype=torch.float32)
        student = student_from_teacher(t32, decoder_layers=2)[0].set_compute("fp32")
        del t32
    else:
        scfg = CONFIGS[c["student"]]
        ws = make_weights(scfg, c["s_seed"], per_tensor=True, embed_std=mg.EMBED_STD)
    s, t, m, grad, batch = _step_f32(scfg, ws, tcfg, wt, feats, dec, lab, c["freeze_encoder"],
                                     c["freeze_embed_positions"], student=student)
    for k, fk in (("loss", "loss"), ("ce_loss", "ce"), ("kl_loss", "kl")):
        ref = float(g["f32|" + fk])
        assert abs(m[k] - ref) / abs(ref) < 2e-5, (k, m[k], ref)
    names = [str(n) for n in g["grad_names"]]
    r = np.abs(_grad_norms(s, grad, names) - g["f32|grad_norms"]) / g["f32|grad_norms"]
    assert r.max() < 1e-3, (names[int(r.argmax())], r.max())
    p0 = "model.decoder.layers.0.fc1.weight"
    o = s.store.offset[p0]
    gsub = grad[o: o + s.store.numel(p0)].view(s.store.segs[p0])[::37, ::29]
    assert rel(gsub, torch.from_numpy(g["f32|grad_dec0_fc1_sub"])) < 1e-4
