"""ORACLE (test infrastructure only): torch-CPU restatement of the Whisper forward
the reference's hot path runs, with the rounding points of CUDA bf16 autocast.

Follows HF Transformers Whisper (HF: = /usr/local/lib/python3.10/dist-packages/
transformers/models/whisper/modeling_whisper.py, 5.15; reference pins 4.45.2 with
the same arithmetic):
  encoder  HF:592-646  conv1/gelu/conv2(stride 2)/gelu + embed_positions, pre-LN
                       layers (HF:379-413), final layer_norm
  decoder  HF:690-797  embed_tokens + embed_positions, causal self-attn,
                       cross-attn, MLP (HF:448-506), final layer_norm
  attention HF:265-350 q_proj * hd^-0.5, k_proj has no bias, softmax(QK^T)V
  head     HF:994-1100 proj_out tied to embed_tokens; CE mean over labels != -100

`amp=True` emulates `Accelerator(mixed_precision="bf16")` (autocast on CUDA,
ACC:accelerator.py:1818-1829): every Linear/Conv1d rounds its inputs, weight and
bias to bf16 and its output to bf16 (fp32 accumulate); LayerNorm / softmax /
cross-entropy run in fp32; residual adds promote (fp32 stream for fp32 params,
bf16 stream for bf16 params such as the teacher, `run_distillation.py:1011-1018`).
Attention under amp follows the flash/SDPA recipe: fp32 scores, P = exp(S - max)
rounded to bf16 for the PV product, normalised by the fp32 row sum, output bf16.
`amp=False` is the plain fp32 model (the golden-vector pin against HF).
`half=torch.float16` (with amp=True, stream_bf16=True) is the torch_dtype=float16 model without autocast
(run_eval.py:99,500-509, run_pseudo_labelling.py:461-463): the same rounding points in fp16 (fp16
weights, Linear / conv / SDPA outputs, residual stream; LayerNorm and GELU computed in fp32, rounded to
fp16; P rounded to fp16 for PV), plus the fp16 encoder-layer clamp (HF:409-411).  Pinned to HF fp16 on
CPU (tests/golden/fp16.npz, tests/test_oracle_golden.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


class Ref:
    """Functional Whisper over an HF-keyed state dict of torch tensors."""

    def __init__(self, cfg: dict, params: dict, amp: bool = False, stream_bf16: bool = False, half=torch.bfloat16):
        self.cfg, self.p, self.amp, self.sbf = cfg, params, amp, stream_bf16
        self.d = cfg["d_model"]
        self.half = half
        self.f16 = half == torch.float16
        self._bf = lambda x: x.to(half).to(torch.float32)       # the 16-bit rounding point

    # -- primitives -------------------------------------------------------
    def lin(self, x, w, b=None):
        if self.amp:
            y = self._bf(x) @ self._bf(w).t()
            if b is not None:
                y = y + self._bf(b)
            return self._bf(y)
        return F.linear(x, w, b)

    def ln(self, x, pfx):
        w, b = self.p[pfx + ".weight"].float(), self.p[pfx + ".bias"].float()
        y = F.layer_norm(x.float(), (self.d,), w, b, 1e-5)
        return self._bf(y) if self.f16 else y

    def gelu(self, x):
        y = F.gelu(x)
        return self._bf(y) if self.amp else y

    def resid(self, r, y):
        out = r + y
        return self._bf(out) if self.sbf else out

    def attn(self, q, k, v, causal):
        """q,k,v [B,H,T,hd] with q already scaled."""
        s = q @ k.transpose(-1, -2)
        if causal:
            Tq, Tk = s.shape[-2], s.shape[-1]
            mask = torch.ones(Tq, Tk, dtype=torch.bool).triu(1 + Tk - Tq)
            s = s.masked_fill(mask, float("-inf"))
        if self.amp:
            m = s.amax(-1, keepdim=True)
            e = torch.exp(s - m)
            l = e.sum(-1, keepdim=True)
            return self._bf((self._bf(e) @ v) / l)
        return torch.softmax(s, -1) @ v

    def mha(self, x, kv, pfx, H, causal):
        B, Tq, d = x.shape
        hd = d // H
        scaling = hd ** -0.5
        q = self.lin(x, self.p[pfx + ".q_proj.weight"], self.p[pfx + ".q_proj.bias"]) * scaling
        k = self.lin(kv, self.p[pfx + ".k_proj.weight"])
        v = self.lin(kv, self.p[pfx + ".v_proj.weight"], self.p[pfx + ".v_proj.bias"])
        Tk = kv.shape[1]
        sh = lambda t, T: t.view(B, T, H, hd).transpose(1, 2)
        o = self.attn(sh(q, Tq), sh(k, Tk), sh(v, Tk), causal)
        o = o.transpose(1, 2).reshape(B, Tq, d)
        return self.lin(o, self.p[pfx + ".out_proj.weight"], self.p[pfx + ".out_proj.bias"])

    def mlp(self, x, pfx):
        h = self.gelu(self.lin(x, self.p[pfx + ".fc1.weight"], self.p[pfx + ".fc1.bias"]))
        return self.lin(h, self.p[pfx + ".fc2.weight"], self.p[pfx + ".fc2.bias"])

    # -- encoder / decoder -------------------------------------------------
    def encoder(self, feats):
        p, H = self.p, self.cfg["encoder_attention_heads"]
        x = feats.float()
        w1, b1 = p["model.encoder.conv1.weight"], p["model.encoder.conv1.bias"]
        w2, b2 = p["model.encoder.conv2.weight"], p["model.encoder.conv2.bias"]
        if self.amp:
            bf = self._bf
            h = bf(F.conv1d(bf(x), bf(w1), bf(b1), padding=1))
            h = self.gelu(h)
            h = bf(F.conv1d(h, bf(w2), bf(b2), stride=2, padding=1))
            h = self.gelu(h)
        else:
            h = F.gelu(F.conv1d(x, w1.float(), b1.float(), padding=1))
            h = F.gelu(F.conv1d(h, w2.float(), b2.float(), stride=2, padding=1))
        h = h.permute(0, 2, 1)
        h = self.resid(p["model.encoder.embed_positions.weight"].float(), h)
        for i in range(self.cfg["encoder_layers"]):
            pf = f"model.encoder.layers.{i}"
            x = self.ln(h, pf + ".self_attn_layer_norm")
            h = self.resid(h, self.mha(x, x, pf + ".self_attn", H, False))
            h = self.resid(h, self.mlp(self.ln(h, pf + ".final_layer_norm"), pf))
            if self.f16:
                h = h.clamp(-64504.0, 64504.0).to(torch.float16).float()
        return self.ln(h, "model.encoder.layer_norm")

    def decoder(self, ids, enc):
        p, H = self.p, self.cfg["decoder_attention_heads"]
        T = ids.shape[1]
        tok = p["model.decoder.embed_tokens.weight"][ids].float()
        pos = p["model.decoder.embed_positions.weight"][:T].float()
        h = self.resid(tok, pos)
        for i in range(self.cfg["decoder_layers"]):
            pf = f"model.decoder.layers.{i}"
            x = self.ln(h, pf + ".self_attn_layer_norm")
            h = self.resid(h, self.mha(x, x, pf + ".self_attn", H, True))
            x = self.ln(h, pf + ".encoder_attn_layer_norm")
            h = self.resid(h, self.mha(x, enc, pf + ".encoder_attn", H, False))
            h = self.resid(h, self.mlp(self.ln(h, pf + ".final_layer_norm"), pf))
        return self.ln(h, "model.decoder.layer_norm")

    def logits(self, hdec):
        return self.lin(hdec, self.p["model.decoder.embed_tokens.weight"]).float()

    def forward(self, feats=None, decoder_input_ids=None, labels=None, enc=None):
        """Mirrors WhisperForConditionalGeneration.forward: returns dict(loss, logits, enc)."""
        if enc is None:
            enc = self.encoder(feats)
        if decoder_input_ids is None:
            from .labels import shift_tokens_right
            decoder_input_ids = torch.from_numpy(shift_tokens_right(labels.numpy(), self.cfg["pad_token_id"],
                                                                    self.cfg["decoder_start_token_id"]))
        hdec = self.decoder(decoder_input_ids, enc)
        lg = self.logits(hdec)
        loss = None
        if labels is not None:
            loss = F.cross_entropy(lg.reshape(-1, lg.shape[-1]), labels.reshape(-1), ignore_index=-100)
        return dict(loss=loss, logits=lg, enc=enc, hdec=hdec)


def to_torch(np_params: dict, dtype=torch.float32, requires_grad=False):
    out = {}
    for k, v in np_params.items():
        t = torch.from_numpy(v).to(dtype)
        if requires_grad:
            t.requires_grad_(True)
        out[k] = t
    return out


def count_flops_per_clip(cfg: dict, T_dec: int = 447, T_enc: int = 1500) -> dict:
    """Algorithmic FLOPs (2*MAC) per clip of one forward, SURVEY.md §8(d) formula."""
    d, V, fe, fd = cfg["d_model"], cfg["vocab_size"], cfg["encoder_ffn_dim"], cfg["decoder_ffn_dim"]
    conv = 2 * (2 * T_enc) * (cfg["num_mel_bins"] * 3) * d + 2 * T_enc * (3 * d) * d
    enc_layer = 2 * T_enc * d * (4 * d) + 2 * 2 * T_enc * d * fe + 2 * 2 * T_enc * T_enc * d
    dec_layer = (2 * T_dec * d * 4 * d + 2 * 2 * T_dec * T_dec * d
                 + 2 * T_dec * d * 2 * d + 2 * T_enc * d * 2 * d + 2 * 2 * T_dec * T_enc * d
                 + 2 * 2 * T_dec * d * fd)
    head = 2 * T_dec * d * V
    return dict(encoder=conv + cfg["encoder_layers"] * enc_layer, decoder=cfg["decoder_layers"] * dec_layer,
                head=head, conv=conv)
