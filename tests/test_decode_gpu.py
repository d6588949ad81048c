"""Greedy KV-cache decoding on the GPU, bf16-autocast path.

* tw_decode_attn vs an fp64 softmax-attention reference (single query row per (b, h), strided
  caches; B*H < 640 over >= 2 chunks of keys runs the split-key variant + combine, B*H >= 640 the
  one-workgroup-per-row kernel; Tk from 1 to 2048, fixed or read from the device step counter);
* tw_greedy_select vs torch (suppress / begin-suppress masks, ties -> lowest id, finished rows);
* generate() KV cache vs a full recompute of the prefix with the same engine (every step);
* generate() under bf16 autocast vs the bf16-autocast oracle (oracle/whisper_ref.Ref(amp=True), pinned to
  HF under autocast by tests/test_oracle_amp_cpu.py) teacher-forced along the emitted sequence: each
  token is the oracle's (rule-processed) argmax or within MARGIN = 0.05 of it -- under one bf16 ulp of
  these |logit| ~ 30 rows -- since both round at the same points but accumulate in different orders.
Token-for-token identity with HF's own greedy ids is the fp32 path's bar (tests/test_fp32_gpu.py: every
fixture reproduced exactly); the autocast path is held to the autocast reference above.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"
MARGIN = 0.05


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("B,H,Tk,dev", [(3, 2, 1, False), (2, 3, 5, False), (4, 20, 447, False), (2, 4, 1500, False),
                                        (1, 1, 2048, False), (1, 20, 1500, False), (13, 20, 1500, False),
                                        (64, 20, 1500, False), (1, 20, 447, True), (40, 20, 200, True)])
def test_decode_attn(B, H, Tk, dev):
    """dev: Tk comes from the device step counter (graph-captured self-attention: Tk = 1 + *tk_dev)."""
    from tw import ops
    g = torch.Generator().manual_seed(B * 131 + Tk)
    d = H * 64
    Tmax = Tk + 3
    cache = bf(torch.randn(B, Tmax, 3 * d, generator=g))          # [q | k | v] rows like the self cache
    t = Tk - 1
    cd = cache.to(DEV)
    flat = cd.view(-1)
    sb = Tmax * 3 * d
    o = torch.empty(B, d, dtype=torch.bfloat16, device=DEV)
    if dev:
        t_dev = torch.tensor([Tk - 1], dtype=torch.int32, device=DEV)
        ops.decode_attn(flat[t * 3 * d:], sb, flat[d:], 3 * d, sb, flat[2 * d:], 3 * d, sb, o, d, B, H, 1, 0.125,
                        tk_dev=t_dev, tk_max=Tmax)
    else:
        ops.decode_attn(flat[t * 3 * d:], sb, flat[d:], 3 * d, sb, flat[2 * d:], 3 * d, sb, o, d, B, H, Tk, 0.125)
    q = cache[:, t, :d].double().view(B, H, 64)
    k = cache[:, :Tk, d:2 * d].double().view(B, Tk, H, 64).transpose(1, 2)
    v = cache[:, :Tk, 2 * d:].double().view(B, Tk, H, 64).transpose(1, 2)
    s = torch.einsum("bhe,bhke->bhk", q, k) * 0.125
    ref = torch.einsum("bhk,bhke->bhe", torch.softmax(s, -1), v).reshape(B, d)
    err = (o.double().cpu() - ref).abs()
    assert err.max() <= 2 ** -7 * ref.abs().max() + 1e-3


@pytest.mark.parametrize("B,H,Tk,dt", [(6, 20, 1500, torch.float16), (5, 2, 1500, torch.bfloat16), (3, 4, 37, torch.float32),
                                       (40, 20, 1500, torch.float16)])
def test_decode_attn_head_strides_shared_kv(B, H, Tk, dt):
    """tw_decode_attn_hs: one clip's head-major K/V ([H][Tk][64] K then V) read by every row of a batch with batch
    stride 0 (the temperature-fallback batch, tw.generation.DecodeSession.set_encoder) == the same rows over B
    copies through tw_decode_attn (B*H one-head clips), bit for bit, on the split (< 640 pairs) and the
    one-workgroup-per-pair kernels."""
    from tw import ops
    g = torch.Generator().manual_seed(B * 7 + Tk)
    q = (torch.randn(B, H * 64, generator=g)).to(dt).to(DEV)
    one = (torch.randn(2 * H * Tk * 64, generator=g)).to(dt).to(DEV)        # K [H][Tk][64] then V
    n1 = H * Tk * 64
    o1 = torch.empty(B, H * 64, dtype=dt, device=DEV)
    ops.decode_attn(q, H * 64, one, 64, 0, one[n1:], 64, 0, o1, H * 64, B, H, Tk, 0.125, hsk=Tk * 64, hsv=Tk * 64)
    # B copies in the B*H one-head-clip form the non-shared head-major path uses
    rep = torch.cat([one[:n1].repeat(B), one[n1:].repeat(B)])
    hv = B * n1
    o2 = torch.empty(B, H * 64, dtype=dt, device=DEV)
    ops.decode_attn(q, 64, rep, 64, Tk * 64, rep[hv:], 64, Tk * 64, o2, 64, B * H, 1, Tk, 0.125)
    assert torch.equal(o1, o2)


@pytest.mark.parametrize("B,Tk,H,dt", [(3, 1500, 20, torch.bfloat16), (2, 7, 2, torch.float32), (1, 1500, 6, torch.bfloat16)])
def test_kv_head_major(B, Tk, H, dt):
    """tw_kv_head_major is the exact permutation [B*Tk][k | v] -> K [B][H][Tk][64], V [B][H][Tk][64] (a padded
    source row stride included), and decode attention over it (B*H one-head clips) equals the row-interleaved
    call bit for bit."""
    from tw import ops
    d = 64 * H
    ld = 2 * d + 8
    src = torch.randn(B * Tk, ld, device=DEV).to(dt)
    dst = torch.full((2 * B * H * Tk * 64,), float("nan"), device=DEV).to(dt)
    ops.kv_head_major(src, ld, dst, B, Tk, H)
    want_k = src[:, :d].reshape(B, Tk, H, 64).transpose(1, 2).reshape(-1)
    want_v = src[:, d:2 * d].reshape(B, Tk, H, 64).transpose(1, 2).reshape(-1)
    half = B * H * Tk * 64
    assert torch.equal(dst[:half], want_k) and torch.equal(dst[half:], want_v)
    q = torch.randn(B, d, device=DEV).to(dt)
    o_row = torch.empty(B, d, device=DEV).to(dt)
    o_hm = torch.empty(B, d, device=DEV).to(dt)
    ops.decode_attn(q, d, src, ld, Tk * ld, src[:, d:], ld, Tk * ld, o_row, d, B, H, Tk, 0.125)
    ops.decode_attn(q, 64, dst, 64, Tk * 64, dst[half:], 64, Tk * 64, o_hm, 64, B * H, 1, Tk, 0.125)
    assert torch.equal(o_row, o_hm)


def test_greedy_select():
    from tw import ops
    g = torch.Generator().manual_seed(7)
    B, V, Vp = 5, 51865, 51904
    logits = bf(torch.randn(B, Vp, generator=g) * 3)
    logits[1, 100] = 50.0                       # suppressed winner -> next best
    logits[2, 220] = 60.0                       # begin-suppressed winner
    logits[3, 7] = 40.0; logits[3, 9] = 40.0    # tie -> lowest id
    logits[:, V:] = 99.0                        # padding columns are never candidates
    sup, beg = [100, 5000], [220, 50257]
    ld = logits.to(DEV)
    done = torch.tensor([0, 0, 0, 0, 1], dtype=torch.uint8, device=DEV)
    ids = torch.zeros(B, 10, dtype=torch.int64, device=DEV)
    nxt = torch.zeros(B, dtype=torch.int64, device=DEV)
    ops.greedy_select(ld, Vp, B, V, ops.token_bitmask(sup, V, DEV), ops.token_bitmask(beg, V, DEV), True, 50257,
                      done, ids, 4, nxt)
    ref = logits[:, :V].float().clone()
    ref[:, sup] = -float("inf")
    ref[:, beg] = -float("inf")
    want = ref.argmax(-1)
    want[4] = 50257
    assert torch.equal(ids[:, 4].cpu(), want) and torch.equal(nxt.cpu(), want)
    assert int(ids[3, 4]) == 7
    assert done.cpu().tolist() == [int(w == 50257) for w in want.tolist()[:4]] + [1]


def _micro(dtype=torch.float32, lin_std=0.2):
    from oracle.weights import CONFIGS, make_weights
    from tw.config import GenerationConfig, WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    cfg = CONFIGS["micro"]
    w = make_weights(cfg, 1, lin_std=lin_std)
    m = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**cfg),
                                                        {k: torch.from_numpy(v) for k, v in w.items()}, dtype=dtype)
    return cfg, w, m, GenerationConfig


def _feats():
    from oracle import logmel
    return torch.from_numpy(logmel.log_mel_batch([logmel.synthetic_clip(0), logmel.synthetic_clip(2, 9.0),
                                                  logmel.synthetic_clip(4, 25.0)]))


def test_generate_cache_matches_full_recompute():
    """Every KV-cache step equals (to bf16 noise) the last-position logits of a full decoder pass."""
    cfg, w, m, GC = _micro()
    g = load_golden("greedy")
    m.generation_config = GC(suppress_tokens=g["suppress"].tolist(), begin_suppress_tokens=[220, 50257])
    prompt = g["greedy_prompt"].tolist()
    feats = _feats()
    gen = m.generate(feats, decoder_input_ids=torch.tensor([prompt] * 3), max_length=40)
    assert gen.shape[1] >= 16
    seq = torch.cat([torch.tensor([prompt] * 3), gen.cpu()], 1)
    out = m(input_features=feats.to(DEV), decoder_input_ids=seq.to(DEV))
    lg = out.logits.float().cpu()
    sup = g["suppress"].tolist()
    P = len(prompt)
    for j in range(gen.shape[1]):
        row = lg[:, P - 1 + j].clone()
        row[:, sup] = -float("inf")
        if j == 0:
            row[:, [220, 50257]] = -float("inf")
        tok = seq[:, P + j]
        live = torch.ones(3, dtype=torch.bool) if j == 0 else (seq[:, P:P + j] != 50257).all(1)
        gap = row.max(-1).values - row.gather(1, tok[:, None])[:, 0]
        assert bool((gap[live] <= MARGIN).all()), (j, gap)


def _teacher_forced(ref, feats, seq):
    with torch.no_grad():
        return ref.logits(ref.decoder(seq[:, :-1], ref.encoder(feats))).float()


def _mask(row, j, sup):
    row = row.clone()
    row[:, sup] = -float("inf")
    if j == 0:
        row[:, [220, 50257]] = -float("inf")
    return row


def test_generate_matches_autocast_oracle():
    """bf16-autocast oracle teacher-forced along the emitted tokens: each token is its argmax or within
    MARGIN of it (same rounding points, different accumulation order)."""
    from oracle.whisper_ref import Ref, to_torch
    cfg, w, m, GC = _micro()
    g = load_golden("greedy")
    sup = g["suppress"].tolist()
    m.generation_config = GC(suppress_tokens=sup, begin_suppress_tokens=[220, 50257])
    prompt = g["greedy_prompt"].tolist()
    P = len(prompt)
    feats = _feats()
    gen = m.generate(feats, decoder_input_ids=torch.tensor([prompt] * 3), max_length=64).cpu()
    assert gen.shape[1] == g["greedy_ids"].shape[1]          # HF's length rule (max_length + P initial tokens)
    seq = torch.cat([torch.tensor([prompt] * 3), gen], 1)
    lg_amp = _teacher_forced(Ref(cfg, to_torch(w), amp=True), feats, seq)
    for j in range(gen.shape[1]):
        live = torch.ones(3, dtype=torch.bool) if j == 0 else (gen[:, :j] != 50257).all(1)
        ra = _mask(lg_amp[:, P - 1 + j], j, sup)
        gap = ra.max(-1).values - ra.gather(1, gen[:, j:j + 1])[:, 0]
        assert bool((gap[live] <= MARGIN).all()), (j, gap)


def test_generate_builds_prompt_and_stops():
    """Prompt from generation_config (language / task / notimestamps) and early stop on eos."""
    from tw.generation import build_prompt
    cfg, w, m, GC = _micro()
    gc = GC(lang_to_id={"<|zh|>": 50260, "<|en|>": 50259})
    assert build_prompt(gc, "zh", "transcribe") == [50258, 50260, 50359, 50363]
    assert build_prompt(gc, "en", "translate") == [50258, 50259, 50358, 50363]
    m.generation_config = gc
    gen = m.generate(_feats()[:2], language="zh", task="transcribe", max_new_tokens=12)
    assert gen.shape[0] == 2 and 1 <= gen.shape[1] <= 12
    # rows that finished are padded with eos
    for r in gen.cpu().tolist():
        if 50257 in r:
            k = r.index(50257)
            assert all(x == 50257 for x in r[k:])


def test_generate_graph_replay_equals_eager():
    """The HIP-graph replay of the position-independent step emits exactly the eager tokens."""
    cfg, w, m, GC = _micro()
    g = load_golden("greedy")
    m.generation_config = GC(suppress_tokens=g["suppress"].tolist(), begin_suppress_tokens=[220, 50257])
    prompt = torch.tensor([g["greedy_prompt"].tolist()] * 3)
    feats = _feats()
    a = m.generate(feats, decoder_input_ids=prompt, max_length=48, use_graph=True).cpu()
    b = m.generate(feats, decoder_input_ids=prompt, max_length=48, use_graph=False).cpu()
    assert torch.equal(a, b)


def _ts_model():
    import os, sys
    import oracle.fixture_inputs as mg
    cfg, w, m, GC = _micro()
    m.generation_config = GC({k: mg.TS_GENERATION[k] for k in mg.TW_GENERATION_KEYS})
    return mg, cfg, w, m


def test_generate_timestamps_short_form():
    """return_timestamps=True on <= 30 s inputs: HF runs its seek loop here too (a window that ends on a timestamp
    pair before the end of the audio is followed by a window from that timestamp: generation_whisper.py:785-898,
    pinned at large-v2 dims by tests/test_lv2_decode_gpu.py).  Every window's tokens obey the HF timestamp rules
    against the bf16-autocast oracle teacher-forced along them (argmax within MARGIN; when the timestamp-mass
    decision itself is within MARGIN either branch is accepted), and the windows follow the seek loop."""
    from oracle.whisper_ref import Ref, to_torch
    mg, cfg, w, m = _ts_model()
    feats = torch.from_numpy(np.stack([_feats()[0].numpy(), _feats()[1].numpy()]))
    trace = []
    gen = m.generate(feats, return_timestamps=True, language="zh", task="transcribe", max_new_tokens=48,
                     _trace=trace).cpu()
    prompt = [50258, 50260, 50359]
    ref = Ref(cfg, to_torch(w), amp=True)
    seen = {0: 0, 1: 0}
    for t in trace:
        b, seek, n = t["b"], t["seek"], t["n"]
        assert t["prompt"] == prompt and n == 3000 - seek
        seen[b] += 1
        seg = torch.zeros(1, 80, 3000)
        seg[0, :, :n] = feats[b, :, seek:seek + n]
        _check_ts_window(ref, seg, prompt, t["raw"], mg.SUPPRESS)
        assert t["raw"][0] >= 50364                       # every window opens on a timestamp
    assert seen[0] >= 1 and seen[1] >= 1
    assert (gen[:, 0] >= 50364).all()


def _either_branch(pre, tok, tol):
    """With the timestamp-mass comparison within noise, tok is the (near-)argmax of the row without
    the mass rule, or — the rule fired — of the timestamps alone (every text id masked)."""
    if float(pre.max() - pre[tok]) <= tol:
        return True
    return tok >= 50364 and float(pre[50364:].max() - pre[tok]) <= tol


def _check_ts_window(ref, feats1, prompt, toks, sup, b=0):
    """bf16-autocast oracle teacher-forced along one window's tokens: each token obeys the HF
    timestamp rules (argmax within 2 bf16 ulps; either branch when the mass rule is a tie)."""
    from oracle import greedy_ref
    P = len(prompt)
    seq = torch.tensor([prompt + toks])
    with torch.no_grad():
        lg = ref.logits(ref.decoder(seq[:, :-1], ref.encoder(feats1))).float()[0]
    for j, tok in enumerate(toks):
        if j > 0 and toks[j - 1] == 50257:
            break
        row = lg[P - 1 + j].clone()
        row[sup] = -float("inf")
        if j == 0:
            row[[220, 50257]] = -float("inf")
        full = greedy_ref.timestamp_rules(row, toks[:j], j == 0, max_initial=50)
        # up to 4 bf16 ulps: hundreds of cached positions accumulate in a different order
        tol = max(MARGIN, 2 ** -6 * float(full.max().abs()))
        ok = float(full.max() - full[tok]) <= tol
        if not ok:
            pre = greedy_ref.timestamp_rules(row, toks[:j], j == 0, max_initial=50, apply_mass=False)
            near = abs(float(pre[50364:].logsumexp(-1)) - float(pre[:50364].max())) <= tol
            ok = near and _either_branch(pre, tok, tol)
        assert ok, (j, tok, float(full.max()), float(full[tok]))


def test_generate_longform_matches_hf():
    """65 s input (6500 frames), sequential 30 s windows.  (1) every window's decode obeys the
    timestamp rules vs the bf16-autocast oracle; (2) the host loop (eos/pad trimming, segment split,
    seek by last timestamp) applied to those window outputs is the oracle's restatement of HF's
    loop (the fp32 path reproduces HF's ids exactly: tests/test_fp32_gpu.py)."""
    from oracle import greedy_ref
    from oracle.whisper_ref import Ref, to_torch
    mg, cfg, w, m = _ts_model()
    g = load_golden("greedy_ts")
    lf = torch.from_numpy(mg.longform_features())
    trace = []
    out = m.generate(lf, attention_mask=torch.ones(1, lf.shape[-1], dtype=torch.long), return_timestamps=True,
                     language="zh", task="transcribe", _trace=trace).cpu()[0].tolist()
    prompt = [50258, 50260, 50359]
    ref = Ref(cfg, to_torch(w), amp=True)
    T = lf.shape[-1]
    seek, rebuilt, win_out = 0, [], []
    for tr in trace:
        assert tr["seek"] == seek
        n = min(3000, T - seek)
        seg = torch.zeros(1, 80, 3000)
        seg[0, :, :n] = lf[0, :, seek:seek + n]
        _check_ts_window(ref, seg, prompt, tr["raw"], mg.SUPPRESS)
        seq = list(tr["raw"])
        if seek + 3000 < T and seq and seq[-1] == 50257:
            seq = seq[:-1]
        segs, off = greedy_ref.retrieve_segment(seq, n)
        win_out.append([t for sgm in segs for t in sgm])
        rebuilt.extend(win_out[-1])
        seek += off if off > 0 else n
    assert seek >= T and rebuilt == out and len(trace) >= 3
