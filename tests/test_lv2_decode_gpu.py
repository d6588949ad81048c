"""Greedy / timestamp / long-form decoding at the REAL whisper-large-v2 dimensions (d 1280, 32 + 32 layers, 20 heads:
the model of BASELINE c4 and c5) against HF Transformers itself.

Fixture: tests/golden/lv2_decode.npz, made by tests/golden/make_golden.py gen_lv2_decode in the build container:
HF WhisperForConditionalGeneration at large-v2 dims with the round-6 decode-parity weights
(oracle/fixture_inputs.lv2_decode_weights(large-v2, seed, v_bias): a soft cross-attention whose value path carries the
attended frames' difference from the mean encoder row -- moderate dynamic range (decoder residual stream max ~25,
logits max ~22), audio-dependent (>= 15 distinct tokens per 48-step row, a different row per clip:
tests/test_oracle_golden.py::test_lv2_fixture_is_input_sensitive), and not chaotic), 4 clips, in three arithmetics:
fp32; torch_dtype=float16 (run_eval.py:99, run_pseudo_labelling.py:461-463); the fp32 model under bf16 autocast
(run_distillation.py:1580-1584, generate_step under the bf16 Accelerator).  The reference's decode calls:
  greedy      generate(decoder_input_ids=[SOT, zh, transcribe, notimestamps], max_new_tokens=48)
              (run_pseudo_labelling.py:917-922 / run_distillation.py:1580-1584, num_beams=1), timestamp tokens
              suppressed (fixture_inputs.LV2_GREEDY_SUPPRESS: HF's seek loop after a timestamp pair is not built)
  timestamps  generate(return_timestamps=True, language="zh", task="transcribe", max_new_tokens=48), one clip per call
  long-form   45 s input (fp32), temperature (0.0,), thresholds that never fire (run_eval.py:659-665 path), per-window
              average log-prob and no-speech probability
plus HF's logits TEACHER-FORCED along HF fp32's greedy tokens in each arithmetic (the 16 largest processed fp32 scores'
ids per step, every arithmetic's raw logits there, the row logsumexp, the processed argmax and its top-2 gap).

Every bound below is computed from the fixture, with constants fixed from CPU evidence before the engine ran on it:
  D(tag)     = rms over the valid (row, step, top-16 id) entries of HF_tag - HF_fp32: the whole effect of the 16-bit
               rounding points on the logits (fixture: fp16 0.038, bf16 0.215);
  O(tag)     = rms of oracle_tag - HF_tag over the same entries, oracle_tag = the CPU restatement of the ENGINE's
               rounding points (oracle/whisper_ref.Ref, stored in the fixture): how far a correct 16-bit rounding
               model that is not HF's own code sits from HF (fixture: fp16 0.73 D, bf16 0.32 D -- the flash-attention
               P roundings relative to each implementation's running maxima, HF's CPU kernel in 512-key blocks, are
               16-bit noise of their own);
  K(tag)     = min(0.9, 1.5 x O(tag) / D(tag)): the engine within 1.5 x the oracle's distance, and in any case closer to
               HF_tag than exact fp32 arithmetic (the engine's fp32 path, = HF fp32 to 1e-4) is;
  TIE(tag)   = 2 x max |HF_tag - HF_fp32| over the same entries: a top-2 gap below it is within what the 16-bit
               rounding points move a logit, so a different choice there is a tie, not an error.
Parity bar:
  * fp32 path: greedy and timestamp token ids IDENTICAL to HF fp32 (north star "token ids bit-exact for greedy
    decode"); long-form: the same windows (seeks), each window's tokens identical to HF's up to the window's first
    step whose HF margin is below FP32_TIE = 2e-3 (the whole window and its gates when it has none; the whole
    recording when no window has one); teacher-forced logits within 0.1 x D(fp16) of HF fp32;
  * fp16 model vs HF torch_dtype=float16, bf16 (fp32 parameters, autocast) vs HF bf16 autocast, teacher-forced through
    the engine's KV-cache decode step (DecodeSession, the kernels generate() replays):
      - rms(engine - HF_tag) <= K(tag) x D(tag): a model missing a rounding point (an fp32 residual stream, unrounded
        Linear outputs) sits at ~D(tag) from HF_tag, as fp32 does;
      - the engine's processed argmax agrees with HF_tag's at >= 90 % of the valid steps, and every step where it
        does not has an HF_tag top-2 gap below TIE(tag);
      - logsumexp per step within TIE(tag) / 2 of HF_tag's;
    and free-running: fp16 greedy, fp16 timestamps and bf16 greedy ids identical to HF's free-running ids of that
    arithmetic up to each row's first step whose HF top-2 gap is below TIE(tag) (timestamps: within the first
    window's kept tokens, where output position = decode step).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"
FP32_TIE = 2e-3
EOT = 50257


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.fixture(scope="module")
def lv2():
    import oracle.fixture_inputs as fx
    from oracle.weights import CONFIGS
    g = load_golden("lv2_decode")
    w = fx.lv2_decode_weights(CONFIGS["large-v2"], int(g["seed"]), g["v_bias"])
    return fx, g, {k: torch.from_numpy(v) for k, v in w.items()}


def _model(lv2, dtype, compute, ts):
    from oracle.weights import CONFIGS
    from tw.config import GenerationConfig, WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    fx, g, w = lv2
    m = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**CONFIGS["large-v2"]), w, dtype=dtype,
                                                        compute=compute)
    if ts:
        m.generation_config = GenerationConfig({k: fx.TS_GENERATION[k] for k in fx.TW_GENERATION_KEYS})
    else:
        m.generation_config = GenerationConfig(suppress_tokens=fx.LV2_GREEDY_SUPPRESS, begin_suppress_tokens=[220, EOT])
    return m


def _greedy(m, g, short):
    prompt = torch.tensor([g["prompt"].tolist()] * short.shape[0])
    return m.generate(torch.from_numpy(short), decoder_input_ids=prompt, max_new_tokens=48).cpu().numpy()


def _timestamps(m, short, dtype):
    return m.generate(torch.from_numpy(short).to(dtype), return_timestamps=True, language="zh", task="transcribe",
                      max_new_tokens=48).cpu().numpy()


def _rows(ids):
    """Timestamp rows -> token lists without padding: the fixture pads with -1, the engine's batched result with
    pad (= eos); a row's own closing eos is dropped from both sides alike."""
    return [[int(t) for t in r if t not in (-1, EOT)] for r in ids]


def _rms(x):
    return float(np.sqrt(np.mean(np.asarray(x, dtype=np.float64) ** 2)))


def _bounds(g, tag):
    """(valid-entry mask [B, S], D(tag), TIE(tag), K(tag)) from the fixture (module docstring)."""
    B, S, _ = g["tf_top_ids"].shape
    valid = np.arange(S)[None, :] < g["tf_len"][:, None]
    d = (g[f"tf_{tag}_vals"] - g["tf_f32_vals"])[valid]
    D = _rms(d)
    otag = "oracle16" if tag == "f16" else "oracleb16"
    O = _rms((g[f"tf_{otag}_vals"] - g[f"tf_{tag}_vals"])[valid]) if tag in ("f16", "b16") else 0.0
    return valid, D, 2.0 * float(np.abs(d).max()), min(0.9, 1.5 * O / D)


def test_lv2_fp32_greedy_timestamps_longform_bit_exact(lv2):
    fx, g, _ = lv2
    short, lf = fx.lv2_features()
    m = _model(lv2, torch.float32, "fp32", ts=False)
    np.testing.assert_array_equal(_greedy(m, g, short), g["f32_greedy_ids"])
    m = _model(lv2, torch.float32, "fp32", ts=True)
    assert _rows(_timestamps(m, short, torch.float32)) == _rows(g["f32_ts_ids"])
    lt = torch.from_numpy(lf)
    trace = []
    got_long = m.generate(lt, attention_mask=torch.ones(1, lt.shape[-1], dtype=torch.long), return_timestamps=True,
                          language="zh", task="transcribe", temperature=(0.0,), logprob_threshold=-1e9,
                          no_speech_threshold=1.0, _trace=trace).cpu().numpy()
    steps = g["f32_long_window_steps"].tolist()
    assert len(trace) == len(steps), ([t["seek"] for t in trace], steps)
    lm = g["f32_long_margin"]
    off, exact = 0, 0
    for w, t in enumerate(trace):
        want = [int(x) for x in g["f32_long_window_ids"][w] if x != -1]
        mw = lm[off:off + steps[w]]
        off += steps[w]
        ties = np.nonzero(mw < FP32_TIE)[0]
        n = int(ties[0]) if len(ties) else len(want)
        got = [int(x) for x in t["raw"]]
        assert got[:n] == want[:n], (w, n, got[:n], want[:n])
        if not len(ties):
            exact += 1
            assert got == want, w
            assert abs(t["avg_logprob"] - float(g["f32_long_avg_logprobs"][w])) <= 1e-4, w
            np.testing.assert_allclose(t["no_speech_prob"], g["f32_long_ns_probs"][w], rtol=1e-4, atol=1e-12)
    print(f"fp32 long-form: {exact}/{len(trace)} windows without an HF margin < {FP32_TIE}, all identical")
    if exact == len(trace):
        np.testing.assert_array_equal(got_long, g["f32_long_ids"])


def _teacher_forced(m, short, prompt, forced, suppress, begin_suppress):
    """The engine's KV-cache decode step (tw.generation.DecodeSession, the kernels generate() captures and replays)
    driven along `forced` [B, S]: per step the raw logits (fp32, [B, S, V]) and the argmax of the processed row
    (suppress tokens every step, the begin tokens at the first) [B, S], both on the host."""
    from tw.generation import DecodeSession
    dev = m.device
    enc16 = m.encode(m.conv_input(torch.from_numpy(short).to(dev, torch.float32)))
    B, S = forced.shape
    Tk = enc16.shape[0] // B
    sess = DecodeSession(m, enc16, B, Tk, len(prompt) + S + 1)
    sess.t_dev.zero_()
    for t in prompt[:-1]:
        sess.cur.fill_(int(t))
        sess.step()
    sess.cur.fill_(int(prompt[-1]))
    V = m.config.vocab_size
    sup = torch.tensor(suppress, device=dev)
    forced_d = torch.from_numpy(np.ascontiguousarray(forced)).to(dev, torch.int64)
    raw, am = [], []
    for t in range(S):
        sess.step()
        lg = sess.logits[:, :V].float()
        raw.append(lg.cpu())
        lg = lg.clone()
        lg[:, sup] = -float("inf")
        if t == 0:
            lg[:, begin_suppress] = -float("inf")
        am.append(lg.argmax(-1))
        sess.cur.copy_(forced_d[:, t])
    torch.cuda.synchronize()
    return torch.stack(raw, 1), torch.stack(am, 1).cpu().numpy()


def _forced_tokens(g):
    """HF fp32's greedy tokens, eos-padded to the 48 teacher-forced steps."""
    ids = g["f32_greedy_ids"]
    return np.pad(ids, ((0, 0), (0, 48 - ids.shape[1])), constant_values=EOT)


def test_lv2_fp32_teacher_forced_logits(lv2):
    """The engine's fp32 decode step along HF fp32's tokens: raw logits at the fixture's ids within 0.1 x D(fp16) of
    HF fp32 (exact fp32 arithmetic in another summation order)."""
    fx, g, _ = lv2
    short, _ = fx.lv2_features()
    m = _model(lv2, torch.float32, "fp32", ts=False)
    raw, am = _teacher_forced(m, short, g["prompt"].tolist(), _forced_tokens(g), fx.LV2_GREEDY_SUPPRESS, [220, EOT])
    valid, D16, _, _ = _bounds(g, "f16")
    vals = torch.gather(raw, -1, torch.from_numpy(g["tf_top_ids"]).long()).numpy()
    err = np.abs(vals - g["tf_f32_vals"])[valid]
    print(f"fp32 teacher-forced: max |engine - HF fp32| {err.max():.2e} (bound {0.1 * D16:.2e})")
    assert err.max() <= 0.1 * D16
    assert (am[valid] == g["tf_f32_argmax"][valid]).all()


@pytest.mark.parametrize("arith", ["fp16", "bf16"])
def test_lv2_16bit_teacher_forced_vs_hf(lv2, arith):
    """fp16 model vs HF torch_dtype=float16; bf16 (fp32 parameters, autocast) vs HF under bf16 autocast, teacher-forced
    along HF fp32's tokens: logit distance, argmax agreement and logsumexp bars of the module docstring."""
    fx, g, _ = lv2
    short, _ = fx.lv2_features()
    dt, tag, otag = (torch.float16, "f16", "oracle16") if arith == "fp16" else (torch.float32, "b16", "oracleb16")
    m = _model(lv2, dt, arith, ts=False)
    raw, am = _teacher_forced(m, short, g["prompt"].tolist(), _forced_tokens(g), fx.LV2_GREEDY_SUPPRESS, [220, EOT])
    del m
    torch.cuda.empty_cache()
    valid, D, TIE, K = _bounds(g, tag)
    vals = torch.gather(raw, -1, torch.from_numpy(g["tf_top_ids"]).long()).numpy()
    hf = g[f"tf_{tag}_vals"]
    rms = _rms((vals - hf)[valid])
    orms = _rms((g[f"tf_{otag}_vals"] - hf)[valid])
    lse = torch.logsumexp(raw, -1).numpy()
    lse_err = float(np.abs(lse - g[f"tf_{tag}_lse"])[valid].max())
    want = g[f"tf_{tag}_argmax"]
    agree = am[valid] == want[valid]
    mism_margin = g[f"tf_{tag}_margin"][valid][~agree]
    hf32_agree = float((g["tf_f32_argmax"][valid] == want[valid]).mean())
    print(f"{arith}: rms(engine - HF) {rms:.4f} = {rms / D:.3f} D (oracle {orms / D:.3f} D; D = {D:.4f}); argmax "
          f"agreement {agree.mean():.3f} (HF fp32 vs HF {arith}: {hf32_agree:.3f}); mismatch gaps "
          f"{np.sort(mismatch_list(mism_margin))} < TIE {TIE:.3f}; max lse err {lse_err:.4f}")
    assert rms <= K * D, (rms, K, D)
    assert agree.mean() >= 0.9, agree.mean()
    assert (mism_margin < TIE).all(), (mism_margin, TIE)
    assert lse_err <= TIE / 2, (lse_err, TIE)


def mismatch_list(x):
    return np.round(np.asarray(x, dtype=np.float64), 4)


def _prefix_equal(got, want, margins, tie, what):
    """Each row's tokens identical up to (not including) its first step whose HF top-2 gap is below `tie`."""
    checked = 0
    for r in range(len(want)):
        mr = margins[r]
        ties = np.nonzero(np.nan_to_num(mr, nan=np.inf) < tie)[0]
        n = min(int(ties[0]) if len(ties) else len(want[r]), len(want[r]))
        assert list(got[r][:n]) == list(want[r][:n]), (what, r, n, list(got[r][:n]), list(want[r][:n]))
        checked += n
    print(f"{what}: identical over the {checked} tokens before each row's first HF gap < {tie:.3f}")


@pytest.mark.parametrize("arith", ["fp16", "bf16"])
def test_lv2_16bit_free_running_vs_hf(lv2, arith):
    """Free-running greedy (fp16 and bf16) and timestamps (fp16: the dtype bench.py --config c5 runs) against HF's
    own free-running ids of that arithmetic, up to each row's first HF near-tie (module docstring)."""
    fx, g, _ = lv2
    short, _ = fx.lv2_features()
    dt, tag = (torch.float16, "f16") if arith == "fp16" else (torch.float32, "b16")
    _, _, TIE, _ = _bounds(g, tag)
    m = _model(lv2, dt, arith, ts=False)
    got = _greedy(m, g, short)
    want = g[f"{tag}_greedy_ids"]
    got = np.pad(got, ((0, 0), (0, max(0, want.shape[1] - got.shape[1]))), constant_values=EOT)
    _prefix_equal(got.tolist(), want.tolist(), g[f"{tag}_greedy_margin"].T, TIE, f"{arith} greedy")
    if arith == "fp16":
        from tw.generation import retrieve_segment
        m = _model(lv2, dt, arith, ts=True)
        trace = []
        ts = m.generate(torch.from_numpy(short).to(dt), return_timestamps=True, language="zh", task="transcribe",
                        max_new_tokens=48, _trace=trace).cpu().numpy()
        # the fixture's rows (one clip per call, -1-padded) and the margins of every decode step, windows in order
        # [step, clip]: output position p comes from decode step p within the first window's kept tokens (the tokens
        # its segments keep, retrieve_segment on the engine's first window of that clip)
        want_ts = [[int(t) for t in r if t != -1] for r in g["f16_ts_ids"]]
        got_ts = [list(map(int, r)) for r in ts]
        kept = []
        for r in range(len(want_ts)):
            w0 = [t["raw"] for t in trace if t["b"] == r and t["seek"] == 0][0]
            seq = w0[:-1] if w0 and w0[-1] == EOT else w0
            kept.append(sum(len(x) for x in retrieve_segment(seq, 3000)[0]))
        _prefix_equal([x[:k] for x, k in zip(got_ts, kept)], [x[:k] for x, k in zip(want_ts, kept)],
                      g["f16_ts_margin"].T, TIE, "fp16 timestamps (first windows)")
