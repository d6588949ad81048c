"""The fp16 arithmetic path: a torch_dtype=float16 model without autocast, the arithmetic of the reference's fp16
decode call sites (training/run_eval.py:99 `--dtype float16` default, :500-509 `model.to(dtype)`, :589
`input_features.to(dtype)`; run_pseudo_labelling.py:461-463 under run-pseudo-labelling.sh:30).

Kernels (tw_gemm_f16 / tw_gemv_f16 / tw_attn_fwd_f16 and the fp16 variants of LayerNorm, decode attention,
selection, embedding) against torch fp32 arithmetic on the same fp16 values, rounded where HF rounds:
  * GEMM outputs within 1 fp16 ulp (fp32 accumulation order only), fused GELU / residual / fp16 clamp;
  * attention (P rounded to fp16 for PV, as SDPA's fp16 flash kernel) within 2 fp16 ulps of the row scale.
End to end against HF Transformers run with torch_dtype=float16 (tests/golden/fp16.npz, make_golden.py gen_fp16):
  * micro forward: encoder output and logits within 2 / 4 fp16 ulps of the row scale;
  * greedy ids, timestamp ids (one window and 65 s long-form) and the conditioned long-form: IDENTICAL to HF
    fp16 generate (no near-tie allowance);
  * per-window average log-probs within 5e-3 of the fp16 oracle teacher-forced along the same tokens and within
    2e-2 of HF (the fp16 sequence-order noise floor, measured on the oracle itself), no-speech within 1e-2 rel.
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"
ULP = 2.0 ** -10          # fp16 unit roundoff x 2 (ulp at [1, 2))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _ulps(got, want, mag=None):
    """|got - want| in fp16 ulps of want (elementwise; ulp of 0 = the smallest normal's).  mag: the magnitude of
    the terms summed into each element (sum |a_k w_k| + |bias|): the fp32 accumulation-order noise of any
    order, 2^-16 * mag (K <= 5120 terms), is forgiven first -- it is many fp16 ulps of a result that cancels to
    near zero, and one fp16 ulp otherwise."""
    got, want = got.double().cpu(), want.double().cpu()
    d = (got - want).abs()
    if mag is not None:
        d = (d - 2.0 ** -16 * mag.double().cpu()).clamp_min(0)
    e = torch.floor(torch.log2(want.abs().clamp_min(2.0 ** -14)))
    return d / 2.0 ** (e - 10)


def _ref_lin(A, W, b):
    """fp16 operands -> (fp16-rounded exact product + bias, term magnitude), in float64 on the device."""
    y = A.double() @ W.double().T + b.double()
    mag = A.double().abs() @ W.double().abs().T + b.double().abs()
    return y.half().float(), mag


def _h(x):
    return x.half().float()


# ------------------------------------------------------------------------------------------ kernels
@pytest.mark.parametrize("M,N,K", [(1, 1280, 1280), (8, 1280, 5120), (100, 3840, 1280), (300, 640, 256),
                                   (512, 1280, 5120), (4480, 1280, 1280), (65536, 1024, 512), (65636, 1024, 512)])
def test_gemm_f16_bias_round(M, N, K):
    """Every routing of tw_gemm_f16 (skinny / skinny split-K, 128x128, sub-round split-K, persistent 256x256):
    fp16 output within 1 ulp of the fp32 product of the same fp16 operands (+ fp16 bias).  (65636, 1024, 512): a
    grid the persistent kernel would take but with a ragged last row block -- the fp16 persistent kernel has
    full-tile epilogues only, so the host must route it to the 128x128 kernel (no write past row M)."""
    from tw import ops
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = (torch.randn(M, K, device=DEV, generator=g)).half()
    W = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).half()
    b = torch.randn(N, device=DEV, generator=g).half()
    C = torch.full((M, N), float("nan"), device=DEV, dtype=torch.float16)
    ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=b, flags=ops.GEMM_ROUND)
    ref, mag = _ref_lin(A, W, b)
    err = _ulps(C.float(), ref, mag)
    assert float(err.max()) <= 1.0, float(err.max())


@pytest.mark.parametrize("M", [1500, 65536])
def test_gemm_f16_gelu_residual_clamp(M):
    """M = 1500: the 128x128 kernel; M = 65536: the persistent kernel's fp16 GELU / residual + clamp epilogues."""
    from tw import ops
    g = torch.Generator(device=DEV).manual_seed(7)
    N, K = 1280, 1280
    A = torch.randn(M, K, device=DEV, generator=g).half()
    W = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).half()
    b = torch.randn(N, device=DEV, generator=g).half()
    y, mag = _ref_lin(A, W, b)
    # bias -> fp16 -> GELU (fp32) -> fp16, with the pre-activation (HF: gelu(fc1(x)) on fp16 tensors)
    H, pre = torch.empty(M, N, device=DEV, dtype=torch.float16), torch.empty(M, N, device=DEV, dtype=torch.float16)
    ops.gemm(A, W, H, M, N, K, lda=K, ldb=K, ldc=N, bias=b, aux=pre, ldaux=N,
             flags=ops.GEMM_ROUND | ops.GEMM_GELU | ops.GEMM_AUX_OUT)
    assert float(_ulps(pre.float(), y, mag).max()) <= 1.0
    gelu = _h(torch.nn.functional.gelu(pre.float()))           # GELU of the kernel's own pre-activation
    assert float(_ulps(H.float(), gelu).max()) <= 1.0
    # residual + the encoder clamp, in place: HF's `residual + hidden_states` of two fp16 tensors (one rounding of
    # the exact sum) then clamp(+-64504) -> fp16(64504) = 64512; the Linear output is the kernel's own (no residual)
    P = torch.empty(M, N, device=DEV, dtype=torch.float16)
    ops.gemm(A, W, P, M, N, K, lda=K, ldb=K, ldc=N, bias=b, flags=ops.GEMM_ROUND)
    res = torch.randn(M, N, device=DEV, generator=g).half()
    res[:8] = 65000.0
    res[8:16] = -65500.0
    X = res.clone()
    ops.gemm(A, W, X, M, N, K, lda=K, ldb=K, ldc=N, bias=b, res=X, ldr=N, flags=ops.GEMM_ROUND | ops.GEMM_CLAMP16)
    want = (P.float() + res.float()).half().float().clamp(-64504.0, 64504.0).half()
    bad = (X.float() != want.float()).nonzero()
    assert bad.shape[0] == 0, (bad.shape[0], bad[:6].tolist(), [(float(X[i, j]), float(want[i, j]), float(P[i, j]),
                                                                float(res[i, j])) for i, j in bad[:6].tolist()])
    assert torch.isfinite(X.float()).all() and (X.float()[:8] > 60000).all() and (X.float()[:16].abs() <= 64512).all()


def test_gemv_f16_layernorm_matches_ln_then_gemm():
    """Batch-1 decode: one tw_gemv_f16 launch (LayerNorm fused) == tw_layernorm_fwd(fp16) + tw_gemm_f16."""
    from tw import ops
    g = torch.Generator(device=DEV).manual_seed(3)
    K, N = 1280, 3840
    x = (torch.randn(2, K, device=DEV, generator=g) * 3).half()
    lw, lb = torch.randn(K, device=DEV, generator=g).half().float(), torch.randn(K, device=DEV, generator=g).half().float()
    W = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).half()
    b = torch.randn(N, device=DEV, generator=g).half()
    y = torch.empty(2, K, device=DEV, dtype=torch.float16)
    ops.layernorm_fwd(x, lw, lb, y)
    ref_ln = _h(torch.nn.functional.layer_norm(x.float(), (K,), lw, lb, 1e-5))
    assert float(_ulps(y.float(), ref_ln).max()) <= 1.0
    C1 = torch.empty(2, N, device=DEV, dtype=torch.float16)
    ops.gemm(y, W, C1, 2, N, K, lda=K, ldb=K, ldc=N, bias=b, flags=ops.GEMM_ROUND)
    C2 = torch.empty(2, N, device=DEV, dtype=torch.float16)
    ops.gemv(x, W, C2, ln_w=lw, ln_b=lb, bias=b, flags=ops.GEMM_ROUND)
    _, mag = _ref_lin(y, W, b)
    assert float(_ulps(C2.float(), C1.float(), 2 * mag).max()) <= 1.0


@pytest.mark.parametrize("B,H,Tq,Tk,causal", [(2, 20, 1500, 1500, False), (2, 4, 447, 447, True),
                                              (1, 20, 447, 1500, False)])
def test_attention_f16(B, H, Tq, Tk, causal):
    from tw import ops
    g = torch.Generator(device=DEV).manual_seed(B + Tq)
    d = H * 64
    q, k, v = (torch.randn(B * T, d, device=DEV, generator=g).half() for T in (Tq, Tk, Tk))
    o = torch.empty(B * Tq, d, device=DEV, dtype=torch.float16)
    ops.attn_fwd(q, d, k, d, v, d, o, d, None, B, H, Tq, Tk, causal, 0.125)
    qq, kk, vv = (t.float().view(B, -1, H, 64).transpose(1, 2) for t in (q, k, v))
    s = (qq @ kk.transpose(-1, -2)) * 0.125
    if causal:
        s = s.masked_fill(torch.ones(Tq, Tk, dtype=torch.bool, device=DEV).triu(1 + Tk - Tq), float("-inf"))
    mx = s.amax(-1, keepdim=True)
    e = torch.exp(s - mx)
    ref = (_h(e) @ vv) / e.sum(-1, keepdim=True)
    ref = _h(ref.transpose(1, 2).reshape(B * Tq, d))
    scale = ref.abs().amax(-1, keepdim=True)
    err = (o.float() - ref).abs() / scale
    assert float(err.max()) <= 2 * ULP, float(err.max())


def test_decode_attention_and_select_f16():
    from tw import ops
    g = torch.Generator(device=DEV).manual_seed(5)
    B, H, Tk = 3, 20, 1500
    q = torch.randn(B, H * 64, device=DEV, generator=g).half()
    kv = torch.randn(B * Tk, 2 * H * 64, device=DEV, generator=g).half()
    o = torch.empty(B, H * 64, device=DEV, dtype=torch.float16)
    ops.decode_attn(q, H * 64, kv, 2 * H * 64, Tk * 2 * H * 64, kv[:, H * 64:], 2 * H * 64, Tk * 2 * H * 64, o, H * 64,
                    B, H, Tk, 0.125)
    K = kv[:, :H * 64].float().view(B, Tk, H, 64).transpose(1, 2)
    V = kv[:, H * 64:].float().view(B, Tk, H, 64).transpose(1, 2)
    p = torch.softmax((q.float().view(B, H, 1, 64) @ K.transpose(-1, -2)) * 0.125, -1)
    ref = _h((p @ V).reshape(B, H * 64))
    assert float(((o.float() - ref).abs() / ref.abs().amax(-1, keepdim=True)).max()) <= 2 * ULP
    # selection on fp16 logits: argmax with suppression, lowest id on ties
    V_ = 51865
    Vp = 51904
    lg = torch.randn(B, Vp, device=DEV, generator=g).half()
    lg[1, 100] = lg[1, 200] = 30.0                       # a tie -> lowest id
    sup = ops.token_bitmask([7, int(lg[0, :V_].float().argmax())], V_, DEV)
    done = torch.zeros(B, dtype=torch.uint8, device=DEV)
    ids = torch.zeros(B, 4, dtype=torch.int64, device=DEV)
    nxt = torch.zeros(B, dtype=torch.int64, device=DEV)
    ops.greedy_select(lg, Vp, B, V_, sup, None, False, 50257, done, ids, 1, nxt)
    ref_l = lg[:, :V_].float().clone()
    ref_l[:, [7, int(lg[0, :V_].float().argmax())]] = -float("inf")
    assert ids[:, 1].tolist() == ref_l.argmax(-1).tolist() and int(ids[1, 1]) == 100
    lp = torch.empty(B, device=DEV)
    ops.token_logprob(lg, Vp, B, V_, 50362, lp)
    assert torch.allclose(lp, torch.log_softmax(lg[:, :V_].float(), -1)[:, 50362], atol=1e-5)


# ------------------------------------------------------------------------------------- end to end
def _model(lin_std=0.02, ts=False):
    from oracle.weights import CONFIGS, make_weights
    from tw.config import GenerationConfig, WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    cfg = CONFIGS["micro"]
    w = make_weights(cfg, 1, lin_std=lin_std)
    m = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**cfg), {k: torch.from_numpy(v) for k, v in
                                                                              w.items()}, dtype=torch.float16)
    assert m.compute == "fp16" and m.act_dtype == torch.float16 and m.store.p16.dtype == torch.float16
    import oracle.fixture_inputs as mg
    if ts:
        m.generation_config = GenerationConfig({k: mg.TS_GENERATION[k] for k in mg.TW_GENERATION_KEYS})
    else:
        m.generation_config = GenerationConfig(suppress_tokens=mg.SUPPRESS, begin_suppress_tokens=[220, 50257])
    return m, mg


def test_fp16_forward_vs_hf():
    g, h = load_golden("micro_step"), load_golden("fp16")
    m, _ = _model()
    feats, dec = torch.from_numpy(g["feats"]).to(DEV), torch.from_numpy(g["dec"]).to(DEV)
    out = m(input_features=feats, decoder_input_ids=dec)
    enc = out.encoder_last_hidden_state.float().cpu().numpy()[:, ::50]
    scale = np.abs(h["f16_enc_sub"]).max(-1, keepdims=True)
    assert (np.abs(enc - h["f16_enc_sub"]) <= 2 * ULP * scale).mean() >= 0.999
    lg = out.logits.float().cpu()
    np.testing.assert_allclose(torch.logsumexp(lg, -1).numpy(), h["f16_s_lse"], rtol=2e-3)
    rows = lg[:, [0, 3, 4, 57, 200, 446], ::97].numpy()
    assert np.abs(rows - h["f16_s_rows"]).max() <= 4 * ULP * np.abs(h["f16_s_rows"]).max()
    assert (lg.argmax(-1).numpy() == h["f16_s_argmax"]).mean() >= 0.99


def test_fp16_greedy_ids_equal_hf():
    h = load_golden("fp16")
    m, mg = _model(lin_std=0.2)
    from test_decode_gpu import _feats
    prompt = torch.tensor([[50258, 50260, 50359, 50363]] * 3)
    for use_graph in (True, False):
        gen = m.generate(_feats(), decoder_input_ids=prompt, max_length=64, use_graph=use_graph).cpu().numpy()
        np.testing.assert_array_equal(gen, h["f16_greedy_ids"])


def test_fp16_timestamps_longform_fallback_vs_hf():
    h = load_golden("fp16")
    m, mg = _model(lin_std=0.2, ts=True)
    from test_decode_gpu import _feats
    feats = _feats()[:2]
    gen = m.generate(feats, return_timestamps=True, language="zh", task="transcribe", max_new_tokens=48).cpu()
    _equal_or_fp32_near_tie(gen.numpy(), h["f16_ts_short_ids"], feats, [50258, 50260, 50359], mg.SUPPRESS)
    lf = torch.from_numpy(mg.longform_features())
    kw = dict(attention_mask=torch.ones(1, lf.shape[-1], dtype=torch.long), return_timestamps=True, language="zh",
              task="transcribe")
    np.testing.assert_array_equal(m.generate(lf, **kw).cpu().numpy(), h["f16_ts_long_ids"])
    cond = m.generate(lf, condition_on_prev_tokens=True, temperature=0.0, **kw).cpu().numpy()
    np.testing.assert_array_equal(cond, h["f16_fb_cond_ids"])
    trace = []
    m.generate(lf, temperature=(0.0,), logprob_threshold=-1e9, no_speech_threshold=1.0, _trace=trace, **kw)
    np.testing.assert_allclose([t["no_speech_prob"] for t in trace], h["f16_fb_ns_probs"], rtol=1e-2)
    # average log-prob over the window's (here 445) tokens.  Against HF: 2e-2.  The fp16 stream makes this mean
    # sensitive to the ORDER of fp32 reductions (one-ulp flips of fp16 activations compound through the layers):
    # the fp16 oracle itself, decoding free-running (the CPU pin, tests/test_oracle_golden.py) and teacher-forced
    # along the same tokens, differs by 1.1e-2 on window 2.  Against that teacher-forced oracle along the
    # engine's own tokens (the same arithmetic; the engine decodes incrementally, so the same order noise applies,
    # measured 0.8-2.4e-3): 5e-3.
    np.testing.assert_allclose([t["avg_logprob"] for t in trace], h["f16_fb_avg_logprobs"], rtol=0, atol=2e-2)
    for t in trace:
        assert abs(t["avg_logprob"] - _oracle_avg(lf, t)) <= 5e-3


def _equal_or_fp32_near_tie(got, want, feats, prompt, suppress):
    """Timestamp ids equal HF fp16's, or each row leaves HF's sequence at a position where the two candidate
    tokens are a near-tie BY THE fp32 REFERENCE: the fp32 oracle (CPU, pinned to HF fp32) teacher-forced along
    HF's prefix puts their processed logits within 2 fp16 ulps of each other (below fp16's own resolution there:
    measured, row 0 token 14 of the short-form fixture: fp32 margin 6.8e-4, both fp16 logits 11.0625 -- an exact
    fp16 tie that HF's CPU kernels broke by lowest id).  After the divergence the row is not compared."""
    from oracle import greedy_ref
    from oracle.weights import CONFIGS, make_weights
    from oracle.whisper_ref import Ref, to_torch
    ref32 = Ref(CONFIGS["micro"], to_torch(make_weights(CONFIGS["micro"], 1, lin_std=0.2)))
    for b in range(want.shape[0]):
        d = np.nonzero(got[b] != want[b])[0]
        if len(d) == 0:
            continue
        j = int(d[0])
        prefix = want[b, :j].tolist()
        with torch.no_grad():
            lg = ref32.forward(feats[b:b + 1].float(), torch.tensor([list(prompt) + prefix]))["logits"][0].float()
        row = lg[len(prompt) - 1 + j].clone()
        row[suppress] = -float("inf")
        if j == 0:
            row[[220, 50257]] = -float("inf")
        r = greedy_ref.timestamp_rules(row, prefix, j == 0, max_initial=50)
        a, c = int(want[b, j]), int(got[b, j])
        ulp = 2.0 ** (np.floor(np.log2(max(abs(float(r[a])), 2.0 ** -14))) - 10)
        margin = abs(float(r[a] - r[c]))
        print(f"row {b} leaves HF fp16 at token {j}: {a} vs {c}, fp32 margin {margin:.2e} ({margin / ulp:.2f} fp16 ulps)")
        assert margin <= 2 * ulp, (b, j, a, c, margin, ulp)


def _oracle_avg(lf, t):
    """The window's average log-prob from the fp16 oracle (CPU), teacher-forced along the engine's tokens."""
    from oracle import greedy_ref
    from oracle.weights import CONFIGS, make_weights
    from oracle.whisper_ref import Ref, to_torch
    import oracle.fixture_inputs as mg
    cfg = CONFIGS["micro"]
    ref = Ref(cfg, to_torch(make_weights(cfg, 1, lin_std=0.2), torch.float16), amp=True, stream_bf16=True,
              half=torch.float16)
    seg = torch.zeros(1, 80, 3000)
    seg[0, :, :t["n"]] = lf[0, :, t["seek"]:t["seek"] + t["n"]]
    raw, P = list(t["raw"]), len(t["prompt"])
    with torch.no_grad():
        lg = ref.forward(seg, torch.tensor([t["prompt"] + raw[:-1]]))["logits"][0].float()
    cand = list(raw)
    while len(cand) > 1 and cand[-1] == 50257 and cand[-2] == 50257:
        cand = cand[:-1]
    scores = []
    for j in range(len(cand)):
        row = lg[P - 1 + j].clone()
        row[mg.SUPPRESS] = -float("inf")
        if j == 0:
            row[[220, 50257]] = -float("inf")
        scores.append(greedy_ref.timestamp_rules(row, raw[:j], j == 0, max_initial=50))
    return greedy_ref.avg_logprob(scores, cand)
