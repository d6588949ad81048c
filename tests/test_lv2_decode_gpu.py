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

Parity bar:
  * fp32 path: token ids IDENTICAL to HF fp32 (north star "token ids bit-exact for greedy decode"); the long-form
    gates within 1e-4 (avg log-prob, absolute) / 1e-4 relative (no-speech probability);
  * fp16 path vs HF fp16 and bf16 path vs HF bf16 autocast: every row identical to HF's up to the first step whose HF
    top-2 margin is below the tie (FP16_TIE 0.05 logits: a few fp16 ulps of the logits; BF16_TIE 0.25: the two engines
    sum K = 1280 / 5120 bf16 products in different orders), after which that row is not compared further; >= 90 % of
    all positions compared, greedy and timestamps alike.
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"
FP16_TIE, BF16_TIE = 0.05, 0.25


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


def _near_tie_compare(got_rows, want_rows, margins, tie):
    """Each row equal to HF's up to the first step whose HF top-2 margin is below `tie`; a row may leave HF's
    sequence only from there on (and is not compared further).  margins[r] = HF's per-step margins of row r, in
    decode order (a timestamp row's output position never runs ahead of its decode step).  -> fraction of the
    HF positions compared."""
    compared = total = 0
    for r, (got, want) in enumerate(zip(got_rows, want_rows)):
        mr = np.asarray(margins[r], dtype=np.float64)
        mr = mr[~np.isnan(mr)]
        ties = np.nonzero(mr < tie)[0]
        first_tie = int(ties[0]) if len(ties) else len(mr)
        total += len(want)
        n = min(len(want), first_tie)
        assert list(got[:n]) == list(want[:n]), (r, first_tie, got[:n], want[:n])
        if first_tie >= len(mr):                       # no near-tie anywhere: the whole row
            assert list(got) == list(want), (r, got, want)
            n = len(want)
        compared += n
    return compared / max(total, 1)


def test_lv2_fp32_greedy_timestamps_longform_bit_exact(lv2):
    mg, g, _ = lv2
    short, lf = mg.lv2_features()
    m = _model(lv2, torch.float32, "fp32", ts=False)
    np.testing.assert_array_equal(_greedy(m, g, short), g["f32_greedy_ids"])
    m = _model(lv2, torch.float32, "fp32", ts=True)
    assert _rows(_timestamps(m, short, torch.float32)) == _rows(g["f32_ts_ids"])
    lt = torch.from_numpy(lf)
    trace = []
    long = m.generate(lt, attention_mask=torch.ones(1, lt.shape[-1], dtype=torch.long), return_timestamps=True,
                      language="zh", task="transcribe", temperature=(0.0,), logprob_threshold=-1e9,
                      no_speech_threshold=1.0, _trace=trace).cpu().numpy()
    np.testing.assert_array_equal(long, g["f32_long_ids"])
    np.testing.assert_allclose([t["avg_logprob"] for t in trace], g["f32_long_avg_logprobs"], rtol=0, atol=1e-4)
    np.testing.assert_allclose([t["no_speech_prob"] for t in trace], g["f32_long_ns_probs"], rtol=1e-4, atol=1e-12)


@pytest.mark.parametrize("arith", ["fp16", "bf16"])
def test_lv2_16bit_greedy_and_timestamps_vs_hf(lv2, arith):
    """fp16 model vs HF torch_dtype=float16, bf16 (autocast) model vs HF under bf16 autocast: the near-tie rule."""
    mg, g, _ = lv2
    short, _ = mg.lv2_features()
    dt, tag, tie = (torch.float16, "f16", FP16_TIE) if arith == "fp16" else (torch.bfloat16, "b16", BF16_TIE)
    m = _model(lv2, dt, arith, ts=False)
    got = _greedy(m, g, short)
    frac = _near_tie_compare([list(r) for r in got], [list(r) for r in g[f"{tag}_greedy_ids"]],
                             g[f"{tag}_greedy_margin"].T, tie)
    assert frac >= 0.9, ("greedy", frac)
    m = _model(lv2, dt, arith, ts=True)
    got = _rows(_timestamps(m, short, torch.float32 if arith == "bf16" else dt))
    want = _rows(g[f"{tag}_ts_ids"])
    frac = _near_tie_compare(got, want, g[f"{tag}_ts_margin"].T, tie)
    assert frac >= 0.9, ("timestamps", frac)
