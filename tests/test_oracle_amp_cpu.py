"""Pin the oracle's bf16-autocast restatement (oracle/whisper_ref.Ref(amp=True), the arithmetic every
GPU parity test of the engine is also compared with) against the reference path itself: HF Whisper's
train_step under bf16 autocast with a bf16 teacher (tests/golden/cfg_c1.npz, amp|..., made by
make_golden.py gen_cfg -- run_distillation.py:1519-1551 with mixed_precision="bf16").

Tolerances as in tests/test_configs_gpu.py: scalars 1e-4 relative (both sides run on this CPU, only
flash-block and accumulation order differ); tensors within 1.5x the reference's own autocast-vs-fp32
distance.  The rounding points themselves are checked layer by layer against HF modules under
torch.autocast: Linear (bf16 inputs, fp32 accumulate, bf16 out) and the attention block.
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import load_golden

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))


def _rl2(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return float((a - b).norm() / b.norm())


def test_oracle_amp_train_step_matches_hf_autocast_c1():
    import make_golden as mg
    from oracle import distill_ref
    from oracle.whisper_ref import Ref, to_torch
    g = load_golden("cfg_c1")
    c = mg.CFG_CASES["c1"]
    scfg, ws, tcfg, wt = mg.cfg_case_weights("c1")
    feats, dec, lab = mg.cfg_case_batch("c1")
    ps = to_torch(ws)
    names = [str(n) for n in g["grad_names"]]
    for n in names:
        ps[n].requires_grad_(True)
    S = Ref(scfg, ps, amp=True)
    T = Ref(tcfg, to_torch(wt, torch.bfloat16), amp=True, stream_bf16=True)
    o = distill_ref.train_step(S, T, torch.from_numpy(feats), torch.from_numpy(dec), torch.from_numpy(lab),
                               share_hidden_states=bool(g["share"]))
    for k, fk in (("loss", "loss"), ("ce_loss", "ce"), ("kl_loss", "kl")):
        ref = float(g["amp|" + fk])
        assert abs(float(o[k]) - ref) / abs(ref) < 1e-4, (k, float(o[k]), ref)
    noise = _rl2(g["amp|s_rows"], g["f32|s_rows"])
    rows = o["s_logits"][:, mg.ROWS, ::mg.VSTRIDE]
    assert _rl2(rows, g["amp|s_rows"]) <= 1.5 * noise
    norms = np.array([ps[n].grad.double().norm().item() for n in names])
    rel = np.abs(norms - g["amp|grad_norms"]) / g["amp|grad_norms"]
    gnoise = np.abs(g["f32|grad_norms"] - g["amp|grad_norms"]) / g["amp|grad_norms"]
    assert rel.max() <= max(1.5 * gnoise.max(), 1e-2), (rel.max(), gnoise.max())


def _hf_model(cfg, w):
    import transformers
    m = transformers.WhisperForConditionalGeneration(transformers.WhisperConfig(**cfg))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()}, strict=False)
    return m


def test_oracle_rounding_points_match_hf_autocast_layer_by_layer():
    """One encoder layer (tiny dims) of HF under CPU bf16 autocast vs the oracle's amp primitives: the
    Linear outputs are identical (same bf16 roundings of inputs / weights, fp32 accumulation, one bf16
    rounding of the output) except where the two fp32 accumulation orders straddle a rounding boundary
    (< 0.2 % of elements, 1 ulp), and the whole layer (LN, attention, GELU MLP, residuals) is within
    half the layer's own autocast-vs-fp32 distance."""
    import make_golden as mg
    from oracle.weights import CONFIGS, make_weights
    from oracle.whisper_ref import Ref, to_torch
    cfg = CONFIGS["tiny"]
    w = make_weights(cfg, 5, per_tensor=True, embed_std=mg.EMBED_STD)
    m = _hf_model(cfg, w)
    ref = Ref(cfg, to_torch(w), amp=True)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, 300, cfg["d_model"], generator=g)
    lay = m.model.encoder.layers[0]
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        q_hf = lay.self_attn.q_proj(x)
        fc1_hf = lay.fc1(x)
    p = "model.encoder.layers.0"
    q_or = ref.lin(x, ref.p[p + ".self_attn.q_proj.weight"], ref.p[p + ".self_attn.q_proj.bias"])
    fc1_or = ref.lin(x, ref.p[p + ".fc1.weight"], ref.p[p + ".fc1.bias"])
    assert q_hf.dtype == torch.bfloat16
    # fp32 accumulation order differs (oneDNN vs torch fp32 matmul of bf16-exact values): the bf16
    # outputs agree exactly except where the fp32 sum straddles a rounding boundary
    for a, b in ((q_hf.float(), q_or), (fc1_hf.float(), fc1_or)):
        diff = (a != b).float().mean().item()
        assert diff < 2e-3, diff
        assert (a - b).abs().max() <= 2 ** -7 * b.abs().max()
    # full encoder layer: HF (autocast) vs oracle amp
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        y_hf = lay(x, attention_mask=None)
        y_hf = y_hf[0] if isinstance(y_hf, tuple) else y_hf
    xl = ref.ln(x, p + ".self_attn_layer_norm")
    h = ref.resid(x, ref.mha(xl, xl, p + ".self_attn", cfg["encoder_attention_heads"], False))
    y_or = ref.resid(h, ref.mlp(ref.ln(h, p + ".final_layer_norm"), p))
    with torch.no_grad():
        y_f32 = lay(x, attention_mask=None)
        y_f32 = y_f32[0] if isinstance(y_f32, tuple) else y_f32
    noise = _rl2(y_hf.float(), y_f32)
    assert _rl2(y_or, y_hf.float()) <= max(0.5 * noise, 1e-4), (_rl2(y_or, y_hf.float()), noise)
