"""Stage-by-stage HIP encoder vs the oracle's autocast restatement (micro config): where does the
encoder output's deviation come from?  Prints relative L2 per stage."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "taiwan-whisper_amd"), os.path.join(REPO, "tests")]

from conftest import load_golden  # noqa: E402
from oracle.weights import CONFIGS, make_weights  # noqa: E402
from oracle.whisper_ref import Ref, to_torch  # noqa: E402
from tw.config import WhisperConfig  # noqa: E402
from tw.modeling import WhisperForConditionalGeneration  # noqa: E402
from tw import ops as F  # noqa: E402


def rl2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


def main():
    cfg = CONFIGS["micro"]
    ws = make_weights(cfg, 1)
    s = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**cfg), {k: torch.from_numpy(v) for k, v in
                                                                               ws.items()}, dtype=torch.float32)
    g = load_golden("micro_step")
    feats = torch.from_numpy(g["feats"])
    ref = Ref(cfg, to_torch(ws), amp=True)
    # oracle stages
    import torch.nn.functional as tf
    from oracle.whisper_ref import _bf
    p = ref.p
    x = feats.float()
    h1 = ref.gelu(_bf(tf.conv1d(_bf(x), _bf(p["model.encoder.conv1.weight"]), _bf(p["model.encoder.conv1.bias"]),
                                padding=1)))
    h2 = ref.gelu(_bf(tf.conv1d(h1, _bf(p["model.encoder.conv2.weight"]), _bf(p["model.encoder.conv2.bias"]),
                                stride=2, padding=1)))
    st0 = ref.resid(p["model.encoder.embed_positions.weight"].float(), h2.permute(0, 2, 1))
    stages_ref = [("conv stem", st0)]
    h = st0
    H = cfg["encoder_attention_heads"]
    for i in range(cfg["encoder_layers"]):
        pf = f"model.encoder.layers.{i}"
        xl = ref.ln(h, pf + ".self_attn_layer_norm")
        h = ref.resid(h, ref.mha(xl, xl, pf + ".self_attn", H, False))
        stages_ref.append((f"layer {i} attn", h))
        h = ref.resid(h, ref.mlp(ref.ln(h, pf + ".final_layer_norm"), pf))
        stages_ref.append((f"layer {i} mlp", h))
    # HIP stages (same calls as WhisperForConditionalGeneration.encode)
    conv_in = s.conv_input(feats.cuda())
    B, T2 = conv_in.shape[0], conv_in.shape[1] - 2
    T, d, nm = T2 // 2, cfg["d_model"], 80
    H1 = torch.zeros(B, T2 + 2, d, dtype=torch.bfloat16, device="cuda")
    gf = F.GEMM_ROUND | F.GEMM_GELU
    F.gemm(conv_in, s._w16("model.encoder.conv1.weight"), H1[:, 1:], T2, d, 3 * nm, lda=nm, ldb=3 * nm, ldc=d,
           batch=B, sA=(T2 + 2) * nm, sC=(T2 + 2) * d, bias=s._w16("model.encoder.conv1.bias"), flags=gf)
    print("conv1 (bf16 after GELU) rel-L2", rl2(H1[:, 1:T2 + 1].float(), h1.permute(0, 2, 1)),
          "exact-match frac", float((H1[:, 1:T2 + 1].float().cpu() == h1.permute(0, 2, 1)).float().mean()))
    xs = torch.empty(B * T, d, dtype=torch.float32, device="cuda")
    F.gemm(H1, s._w16("model.encoder.conv2.weight"), xs, T, d, 3 * d, lda=2 * d, ldb=3 * d, ldc=d, batch=B,
           sA=(T2 + 2) * d, sC=T * d, bias=s._w16("model.encoder.conv2.bias"),
           res=s.store.v32("model.encoder.embed_positions.weight"), ldr=d, res_mod=T, flags=gf)
    hs = [("conv stem", xs.view(B, T, d).clone())]
    xcur = xs
    for i in range(cfg["encoder_layers"]):
        pf = f"model.encoder.layers.{i}"
        xcur, pend = s._attn_block(xcur, pf + ".self_attn", B, T, False)
        if pend is not None:                 # deferred residual update: apply it for the stage dump
            xcur = xcur + pend.float()
        hs.append((f"layer {i} attn", xcur.view(B, T, d).clone()))
        xcur, pend = s._mlp_block(xcur, pf)
        if pend is not None:
            xcur = xcur + pend.float()
        hs.append((f"layer {i} mlp", xcur.view(B, T, d).clone()))
    for (n, a), (_, b) in zip(hs, stages_ref):
        print(f"{n:14s} rel-L2 {rl2(a, b):.3e}")


if __name__ == "__main__":
    main()
