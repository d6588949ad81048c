"""Greedy / timestamp / long-form decoding at the REAL whisper-large-v2 dimensions (d 1280, 32 + 32 layers, 20 heads:
the model of BASELINE c4 and c5) against HF Transformers itself.

Fixture: tests/golden/lv2_decode.npz, made by tests/golden/make_golden.py gen_lv2_decode in the build container:
HF WhisperForConditionalGeneration at large-v2 dims with the documented decode-parity weights
(oracle/weights.lv2_decode_weights(large-v2, seed): the decoder's cross-attention and positions strengthened so that
decoding depends on the audio -- round 4's default-scale weights produced 2-3 distinct tokens per row, the same for every
clip; tests/test_oracle_golden.py::test_lv2_fixture_is_input_sensitive pins that it no longer does), 4 clips, in three
arithmetics: fp32; torch_dtype=float16 (run_eval.py:99, run_pseudo_labelling.py:461-463); the fp32 model under bf16
autocast (run_distillation.py:1580-1584, generate_step under the bf16 Accelerator).  The reference's decode calls:
  greedy      generate(decoder_input_ids=[SOT, zh, transcribe, notimestamps], max_new_tokens=48)
              (run_pseudo_labelling.py:917-922 / run_distillation.py:1580-1584, num_beams=1)
  timestamps  generate(return_timestamps=True, language="zh", task="transcribe", max_new_tokens=48), one clip per call
  long-form   45 s input (fp32), temperature (0.0,), thresholds that never fire (run_eval.py:659-665 path), per-window
              average log-prob and no-speech probability
plus, per decode step and row, HF's margin between the two largest processed scores.

The fixture's dynamic range: the strengthened cross-attention drives the decoder's residual stream to ~2.4e3 and the
logits to ~85 (top-2 margins: median 2.5 logits), so rounding noise is large in absolute terms -- HF's own fp16 and
bf16 greedy rows leave HF's fp32 rows within 0-18 steps, and HF fp32 meets top-2 margins of 1e-3 in the long-form
windows (about 130 fp32 ulps of an 85 logit; the engine and HF sum the same products in different orders).

Parity bar:
  * fp32 path: greedy and timestamp token ids IDENTICAL to HF fp32 (north star "token ids bit-exact for greedy
    decode"); long-form: the same windows (seeks), and each window's tokens identical to HF's up to the window's first
    step whose HF margin is below FP32_TIE = 2e-3 (the whole window when it has none, then its gates within 1e-4
    absolute / 1e-4 relative); measured: the windows with margins of 1.0e-3 and 1.1e-3 are the ones that part;
  * fp16 vs HF fp16 and bf16 (fp32 parameters under autocast) vs HF bf16 autocast, teacher-forced along HF's own
    greedy sequence through the engine's KV-cache decode step (the kernels generate() replays): the engine's argmax
    agrees with HF's token at least as often as exact fp32 arithmetic does -- the engine's fp32 path, bit-exact with
    HF fp32, teacher-forced along the same tokens -- less 5 points, and every engine mismatch sits at an HF margin
    within 1.25x the largest margin at which the fp32 reference itself leaves HF's token (the noise scale of that
    arithmetic on this fixture).  Measured: fp16 157/192 agree (fp32 reference 159), largest mismatch margin 2.69
    (reference 2.94); bf16 120/192 (reference 125), 9.5 (reference 8.0).
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"
FP32_TIE = 2e-3


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _mg():
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    if here not in sys.path:
        sys.path.insert(0, here)
    import make_golden as mg
    return mg


@pytest.fixture(scope="module")
def lv2():
    from oracle.weights import CONFIGS, lv2_decode_weights
    mg = _mg()
    g = load_golden("lv2_decode")
    w = lv2_decode_weights(CONFIGS["large-v2"], int(g["seed"]))
    return mg, g, {k: torch.from_numpy(v) for k, v in w.items()}


def _model(lv2, dtype, compute, ts):
    from oracle.weights import CONFIGS
    from tw.config import GenerationConfig, WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    mg, g, w = lv2
    m = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**CONFIGS["large-v2"]), w, dtype=dtype,
                                                        compute=compute)
    if ts:
        gc = mg.ts_generation_config().to_dict()
        m.generation_config = GenerationConfig({k: gc[k] for k in (
            "decoder_start_token_id", "eos_token_id", "pad_token_id", "suppress_tokens", "begin_suppress_tokens",
            "max_length", "no_timestamps_token_id", "is_multilingual", "lang_to_id", "task_to_id",
            "max_initial_timestamp_index")})
    else:
        m.generation_config = GenerationConfig(suppress_tokens=mg.SUPPRESS, begin_suppress_tokens=[220, 50257])
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
    return [[int(t) for t in r if t not in (-1, 50257)] for r in ids]


def test_lv2_fp32_greedy_timestamps_longform_bit_exact(lv2):
    mg, g, _ = lv2
    short, lf = mg.lv2_features()
    m = _model(lv2, torch.float32, "fp32", ts=False)
    np.testing.assert_array_equal(_greedy(m, g, short), g["f32_greedy_ids"])
    m = _model(lv2, torch.float32, "fp32", ts=True)
    assert _rows(_timestamps(m, short, torch.float32)) == _rows(g["f32_ts_ids"])
    lt = torch.from_numpy(lf)
    trace = []
    m.generate(lt, attention_mask=torch.ones(1, lt.shape[-1], dtype=torch.long), return_timestamps=True,
               language="zh", task="transcribe", temperature=(0.0,), logprob_threshold=-1e9, no_speech_threshold=1.0,
               _trace=trace)
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
    assert exact >= len(trace) // 2, exact


def _teacher_forced_argmax(m, short, prompt, forced, suppress, begin_suppress):
    """The engine's KV-cache decode step (tw.generation.DecodeSession, the kernels generate() captures and replays)
    driven along `forced` [B, S]: per step the argmax of the processed logits (suppress tokens every step, the begin
    tokens at the first) -> [B, S] (host)."""
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
    out = []
    for t in range(S):
        sess.step()
        lg = sess.logits[:, :V].float()
        lg[:, sup] = -float("inf")
        if t == 0:
            lg[:, begin_suppress] = -float("inf")
        out.append(lg.argmax(-1))
        sess.cur.copy_(forced_d[:, t])
    torch.cuda.synchronize()
    return torch.stack(out, 1).cpu().numpy()


@pytest.mark.parametrize("arith", ["fp16", "bf16"])
def test_lv2_16bit_greedy_vs_hf(lv2, arith):
    """fp16 model vs HF torch_dtype=float16; bf16 (fp32 parameters, autocast) vs HF under bf16 autocast: teacher-forced
    agreement with HF's tokens at least that of exact fp32 arithmetic (the engine's fp32 path) less 5 points, every
    mismatch within the fp32 reference's own noise scale (module docstring)."""
    mg, g, _ = lv2
    short, _ = mg.lv2_features()
    dt, tag = (torch.float16, "f16") if arith == "fp16" else (torch.float32, "b16")
    want = g[f"{tag}_greedy_ids"]
    margin = g[f"{tag}_greedy_margin"].T                            # [row, step]
    args = (short, g["prompt"].tolist(), want, mg.SUPPRESS, [220, 50257])
    m = _model(lv2, dt, arith, ts=False)
    tf = _teacher_forced_argmax(m, *args)
    del m
    torch.cuda.empty_cache()
    tf32 = _teacher_forced_argmax(_model(lv2, torch.float32, "fp32", ts=False), *args)
    torch.cuda.empty_cache()
    agree = agree32 = total = 0
    mism, mism32 = [], []
    for r in range(want.shape[0]):
        row = want[r].tolist()
        n = row.index(50257) + 1 if 50257 in row else len(row)     # up to and including the row's own eos
        for t in range(n):
            total += 1
            if tf[r, t] == want[r, t]:
                agree += 1
            else:
                mism.append(float(margin[r, t]))
            if tf32[r, t] == want[r, t]:
                agree32 += 1
            else:
                mism32.append(float(margin[r, t]))
    print(f"{arith}: teacher-forced agreement with HF {agree}/{total} (fp32 reference {agree32}/{total}); "
          f"mismatch HF margins max {max(mism, default=0):.3f} (fp32 reference {max(mism32, default=0):.3f})")
    assert agree >= agree32 - 0.05 * total, (arith, agree, agree32, total)
    assert max(mism, default=0.0) <= 1.25 * max(mism32, default=0.0), (arith, sorted(mism), sorted(mism32))
