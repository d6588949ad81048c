"""Checkpoint layout / resume helpers without a GPU (tw/checkpoint.py vs run_distillation.py).

* HF parameter order and the reference's two optimizer groups are checked against a real
  transformers WhisperForConditionalGeneration (the reference builds its optimizer from
  `student_model.named_parameters()`, run_distillation.py:1434-1449, with get_parameter_names
  :779-795 restated here over the torch module tree).
* Directory naming / rotation / last-checkpoint / skip-batch arithmetic follow :730-774, :1607-1640.
"""
import os

import pytest
import torch

from oracle.weights import CONFIGS


def _hf(cfg):
    import transformers
    return transformers.WhisperForConditionalGeneration(transformers.WhisperConfig(**cfg))


def _reference_parameter_names(model, forbidden_layer_types, forbidden_module=None):
    """run_distillation.py:779-795 behaviour: recurse over named_children, drop parameters of
    forbidden layer types / modules, keep the module's own parameters."""
    result = []
    for name, child in model.named_children():
        if (forbidden_module is None or child not in forbidden_module) and not isinstance(child, tuple(forbidden_layer_types)):
            result += [f"{name}.{n}" for n in _reference_parameter_names(child, forbidden_layer_types, forbidden_module)]
    result += list(model._parameters.keys())
    return result


@pytest.mark.parametrize("name,enc_layers,dec_layers", [("micro", None, None), ("micro", 3, 1)])
def test_hf_parameter_order(name, enc_layers, dec_layers):
    from tw.checkpoint import hf_parameter_names
    from tw.config import WhisperConfig
    cfg = dict(CONFIGS[name])
    if enc_layers:
        cfg.update(encoder_layers=enc_layers, decoder_layers=dec_layers)
    hf = [n for n, _ in _hf(cfg).named_parameters()]
    assert hf_parameter_names(WhisperConfig(**cfg)) == hf


@pytest.mark.parametrize("freeze_encoder,freeze_decoder", [(True, False), (False, False), (True, True)])
def test_optimizer_groups_match_reference_construction(freeze_encoder, freeze_decoder):
    from tw.checkpoint import optimizer_groups
    from tw.config import WhisperConfig
    cfg = CONFIGS["micro"]
    m = _hf(cfg)
    forbidden = []
    if freeze_encoder:
        forbidden.append(m.model.encoder)
    if freeze_decoder:
        forbidden.append(m.model.decoder)
    decay = _reference_parameter_names(m, [torch.nn.LayerNorm], forbidden_module=forbidden)
    decay = set(n for n in decay if "bias" not in n)
    ref0 = [n for n, _ in m.named_parameters() if n in decay]
    ref1 = [n for n, _ in m.named_parameters() if n not in decay]
    g0, g1 = optimizer_groups(WhisperConfig(**cfg), freeze_encoder, freeze_decoder)
    assert (g0, g1) == (ref0, ref1)


def test_checkpoint_naming_rotation_and_last(tmp_path):
    from tw import checkpoint as C
    for step, ep in ((100, 0), (300, 1), (200, 0), (1000, 3)):
        os.makedirs(tmp_path / C.checkpoint_name(step, ep))
    os.makedirs(tmp_path / "runs")
    (tmp_path / "checkpoint-5000-epoch-9.txt").write_text("not a dir")
    assert [os.path.basename(p) for p in C.sorted_checkpoints(tmp_path)] == [
        "checkpoint-100-epoch-0", "checkpoint-200-epoch-0", "checkpoint-300-epoch-1", "checkpoint-1000-epoch-3"]
    assert os.path.basename(C.get_last_checkpoint(tmp_path)) == "checkpoint-1000-epoch-3"
    assert C.parse_checkpoint(C.get_last_checkpoint(tmp_path)) == (1000, 3)
    assert C.rotate_checkpoints(None, tmp_path) == [] and C.rotate_checkpoints(0, tmp_path) == []
    gone = C.rotate_checkpoints(2, tmp_path)
    assert [os.path.basename(p) for p in gone] == ["checkpoint-100-epoch-0", "checkpoint-200-epoch-0"]
    assert [os.path.basename(p) for p in C.sorted_checkpoints(tmp_path)] == [
        "checkpoint-300-epoch-1", "checkpoint-1000-epoch-3"]
    assert C.get_last_checkpoint(tmp_path / "runs") is None
    with pytest.raises(ValueError):
        C.parse_checkpoint("/x/step-3")


def test_resume_skip_batches():
    from tw.checkpoint import resume_skip_batches
    # 250 optimizer steps done, 100 steps per epoch -> 2 epochs done, 50 steps into the third
    assert resume_skip_batches(250, 2, 100, accum=4, streaming=False, max_steps=-1) == 200
    assert resume_skip_batches(250, 2, 100, accum=1, streaming=True, max_steps=-1) is None
    assert resume_skip_batches(250, 2, 100, accum=1, streaming=False, max_steps=1000) is None


@pytest.mark.parametrize("freeze_encoder,freeze_decoder", [(True, False), (False, False), (True, True)])
def test_weight_decay_runs_follow_reference_groups(freeze_encoder, freeze_decoder):
    """The AdamW launches' per-range weight decay (tw.distill.weight_decay_runs over the packed flat
    store) equals the group each parameter sits in inside the reference's torch AdamW
    (run_distillation.py:1424-1456, rebuilt here from an HF module tree), so the update and the
    optimizer.bin groups agree -- incl. freeze_decoder, where the trainable embed_tokens lives under a
    forbidden module and gets weight_decay 0."""
    from tw.config import WhisperConfig
    from tw.distill import set_trainable_like_reference, weight_decay_runs
    from tw.modeling import WhisperForConditionalGeneration
    cfg = CONFIGS["micro"]
    m = _hf(cfg)
    forbidden = [x for x, f in ((m.model.encoder, freeze_encoder), (m.model.decoder, freeze_decoder)) if f]
    decay = set(n for n in _reference_parameter_names(m, [torch.nn.LayerNorm], forbidden_module=forbidden)
                if "bias" not in n)
    s = WhisperForConditionalGeneration(WhisperConfig(**cfg), device="cpu")
    set_trainable_like_reference(s, freeze_encoder, freeze_decoder, True)
    s.pack_for_training()
    runs = weight_decay_runs(s, 0.01, freeze_encoder, freeze_decoder)
    assert all(runs[i][1] <= runs[i + 1][0] for i in range(len(runs) - 1))
    assert runs[0][0] == 0 and runs[-1][1] <= s.train_prefix
    checked = 0
    for n in s.train_names:
        if n.endswith(".zero_bias"):
            continue
        o = s.store.offset[n]
        wd = [w for lo, hi, w in runs if lo <= o < hi]
        assert len(wd) == 1, n
        assert wd[0] == (0.01 if n in decay else 0.0), (n, wd[0])
        checked += 1
    assert checked == len(s.trainable)
    if freeze_decoder:
        assert "model.decoder.embed_tokens.weight" in s.trainable and "model.decoder.embed_tokens.weight" not in decay
