"""fp16 distillation host logic (run_distillation.py:815-817 --dtype float16 -> mixed_precision="fp16"): the loss
scaler's update rule against torch's own (torch._amp_update_scale_, what GradScaler.update runs), the --dtype
mapping, and the fp16-autocast model mode (fp32 master + fp16 weight copy)."""
import pytest
import torch


@pytest.mark.parametrize("interval", [1, 3, 2000])
def test_grad_scaler_update_matches_torch(interval):
    from tw.distill import GradScaler
    ours = GradScaler(growth_interval=interval)
    scale = torch.full((1,), 65536.0)
    tracker = torch.zeros(1, dtype=torch.int32)
    flags = [0, 0, 0, 1, 0, 1, 1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0]
    for f in flags:
        ours.update(bool(f))
        torch._amp_update_scale_(scale, tracker, torch.full((1,), float(f)), 2.0, 0.5, interval)
        assert ours.scale == float(scale.item()) and ours.growth_tracker == int(tracker.item())
    st = ours.state_dict()
    other = GradScaler()
    other.load_state_dict(st)
    assert other.state_dict() == st


def test_grad_scaler_defaults_are_torchs():
    from tw.distill import GradScaler
    ref = torch.amp.GradScaler("cpu")
    ours = GradScaler()
    assert ours.scale == ref.get_scale() and ours.growth_interval == ref.get_growth_interval()
    assert ours.growth_factor == ref.get_growth_factor() and ours.backoff_factor == ref.get_backoff_factor()


def test_dtype_flag_and_fp16_autocast_model():
    from oracle.weights import CONFIGS
    from tw.config import WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    from tw.run_distillation import teacher_dtype
    assert teacher_dtype("float16") == torch.float16 and teacher_dtype("bfloat16") == torch.bfloat16
    with pytest.raises(ValueError):
        teacher_dtype("int8")
    cfg = WhisperConfig(**CONFIGS["micro"])
    m = WhisperForConditionalGeneration(cfg, dtype=torch.float32, device="cpu", compute="fp16")
    assert m.compute == "fp16" and m.act_dtype == torch.float16 and m.stream_dtype == torch.float32
    assert m.store.p16.dtype == torch.float16 and m.store.p32 is not None
    t = WhisperForConditionalGeneration(cfg, dtype=torch.float16, device="cpu")
    assert t.compute == "fp16" and t.stream_dtype == torch.float16
    with pytest.raises(ValueError):
        WhisperForConditionalGeneration(cfg, dtype=torch.bfloat16, device="cpu", compute="fp16")
    with pytest.raises(ValueError):
        t.set_compute("bf16")
