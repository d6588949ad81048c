"""Beam search (`training/run_eval.py:144-147` --num_beams,
`training/run_distillation.py:1476-1484` generation_num_beams) on the GPU engine.

* fp32 path: token-for-token identical to HF 5.15 `generate(num_beams=k)` (GenerationMixin._beam_search) on the
  micro model, k = 2 and 4, for the greedy fixture's weights (every beam runs to max_length) and for the same weights
  with the <|endoftext|> embedding row scaled by 6 (beams finish at different steps, the kept-hypotheses path);
  fixture tests/golden/beam.npz from tests/golden/make_golden.py gen_beam;
* bf16 path: the same call runs; finished rows are padded with eos, and k = 1 is the greedy decode.
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


def test_beam_rejects_timestamps():
    from test_decode_gpu import _feats
    m = _model(1.0, "bf16")
    with pytest.raises(NotImplementedError):
        m.generate(_feats(), num_beams=2, return_timestamps=True)
