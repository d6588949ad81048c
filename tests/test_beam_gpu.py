"""Beam search (`training/run_eval.py:144-147` --num_beams,
`training/run_distillation.py:1476-1484` generation_num_beams) on the GPU engine.

* fp32 path: token-for-token identical to HF 5.15 `generate(num_beams=k)` (GenerationMixin._beam_search) on the
  micro model, k = 2 and 4, for the greedy fixture's weights (every beam runs to max_length) and for the same weights
  with the <|endoftext|> embedding row scaled by 6 (beams finish at different steps, the kept-hypotheses path);
  fixture tests/golden/beam.npz from tests/golden/make_golden.py gen_beam;
* bf16 path: the same call runs; finished rows are padded with eos, and k = 1 is the greedy decode;
* with timestamps (short-form seek loop and long-form, HF generate_with_fallback keeping num_beams at temperature 0):
  fp32 token ids identical to HF and the per-window gates within 1e-4 (tests/golden/beam_ts.npz).
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


def _model(eos_scale, compute):
    from oracle.weights import CONFIGS, make_weights
    from tw.config import GenerationConfig, WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    cfg = CONFIGS["micro"]
    w = make_weights(cfg, 1, lin_std=0.2)
    w["model.decoder.embed_tokens.weight"] = w["model.decoder.embed_tokens.weight"].copy()
    w["model.decoder.embed_tokens.weight"][50257] *= eos_scale
    m = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**cfg),
                                                        {k: torch.from_numpy(v) for k, v in w.items()},
                                                        dtype=torch.float32)
    if compute == "fp32":
        m.set_compute("fp32")
    g = load_golden("greedy")
    m.generation_config = GenerationConfig(suppress_tokens=g["suppress"].tolist(), begin_suppress_tokens=[220, 50257])
    return m


@pytest.mark.parametrize("nb", [2, 4])
@pytest.mark.parametrize("tag,scale", [("", 1.0), ("_eos6", 6.0)])
def test_fp32_beam_bit_exact_vs_hf(nb, tag, scale):
    from test_decode_gpu import _feats
    g = load_golden("beam")
    assert float(g["beam_eos_scale"]) == 6.0
    m = _model(scale, "fp32")
    prompt = torch.tensor([g["beam_prompt"].tolist()] * 3)
    gen = m.generate(_feats(), decoder_input_ids=prompt, max_length=64, num_beams=nb).cpu().numpy()
    np.testing.assert_array_equal(gen, g[f"beam{nb}{tag}_ids"])


def test_bf16_beam_runs_and_pads():
    from test_decode_gpu import _feats
    g = load_golden("beam")
    m = _model(6.0, "bf16")
    prompt = torch.tensor([g["beam_prompt"].tolist()] * 3)
    gen = m.generate(_feats(), decoder_input_ids=prompt, max_length=64, num_beams=4).cpu()
    assert gen.shape[0] == 3 and 1 <= gen.shape[1] <= 64
    for r in gen.tolist():
        if 50257 in r:
            k = r.index(50257)
            assert all(x == 50257 for x in r[k:])
    one = m.generate(_feats(), decoder_input_ids=prompt, max_length=64, num_beams=1).cpu()
    greedy = m.generate(_feats(), decoder_input_ids=prompt, max_length=64).cpu()
    assert torch.equal(one, greedy)


@pytest.mark.parametrize("nb", [2, 4])
def test_fp32_beam_timestamps_longform_bit_exact_vs_hf(nb):
    """num_beams with timestamps (HF generate_with_fallback: the temperature-0 attempt keeps num_beams): the
    short-form seek loop over 2 clips and the 65 s long-form input, token ids identical to HF fp32; the long-form
    windows' gates (average log-prob of the chosen hypothesis's processed scores, no-speech probability) within
    1e-4.  Fixture tests/golden/beam_ts.npz (make_golden.py gen_beam_ts)."""
    from test_decode_gpu import _feats, _ts_model
    mg, cfg, w, m = _ts_model()
    m.set_compute("fp32")
    g = load_golden("beam_ts")
    feats = torch.from_numpy(np.stack([_feats()[0].numpy(), _feats()[1].numpy()]))
    gen = m.generate(feats, return_timestamps=True, language="zh", task="transcribe", max_new_tokens=48,
                     num_beams=nb).cpu().numpy()
    np.testing.assert_array_equal(gen, g[f"bts{nb}_short_ids"])
    lf = torch.from_numpy(mg.longform_features())
    trace = []
    out = m.generate(lf, attention_mask=torch.ones(1, lf.shape[-1], dtype=torch.long), return_timestamps=True,
                     language="zh", task="transcribe", num_beams=nb, temperature=(0.0,), logprob_threshold=-1e9,
                     no_speech_threshold=1.0, _trace=trace).cpu().numpy()
    np.testing.assert_array_equal(out, g[f"bts{nb}_long_ids"])
    np.testing.assert_allclose([t["avg_logprob"] for t in trace], g[f"bts{nb}_long_avg_logprobs"], rtol=0, atol=1e-4)
    np.testing.assert_allclose([t["no_speech_prob"] for t in trace], g[f"bts{nb}_long_ns_probs"], rtol=1e-4,
                               atol=1e-12)


def test_bf16_beam_timestamps_runs():
    """bf16 path: num_beams with timestamps decodes every window opening on a timestamp, timestamps within a window
    never decreasing; num_beams=1 is the greedy timestamp decode."""
    from test_decode_gpu import _feats, _ts_model
    mg, cfg, w, m = _ts_model()
    feats = torch.from_numpy(np.stack([_feats()[0].numpy(), _feats()[1].numpy()]))
    trace = []
    gen = m.generate(feats, return_timestamps=True, language="zh", task="transcribe", max_new_tokens=48, num_beams=3,
                     _trace=trace).cpu()
    assert gen.shape[0] == 2 and (gen[:, 0] >= 50364).all()
    for t in trace:
        ts = [x for x in t["raw"] if x >= 50364]
        assert ts and t["raw"][0] >= 50364 and ts == sorted(ts), t["raw"]
    kw = dict(return_timestamps=True, language="zh", task="transcribe", max_new_tokens=48)
    assert torch.equal(m.generate(feats, num_beams=1, **kw).cpu(), m.generate(feats, **kw).cpu())
