"""ORACLE (test infrastructure only): Whisper configs and a documented PRNG weight
generator used by the parity tests and golden fixtures.

Configs mirror the HF `WhisperConfig` fields the reference reads
(HF:models/whisper/configuration_whisper.py; real checkpoint special ids per
SURVEY.md Appendix A: decoder_start 50258, pad = eos = bos = 50257).

Weight recipe (numpy PCG64, documented so any side can regenerate it):
  rng = np.random.Generator(np.random.PCG64(seed)); tensors are drawn in the
  sorted order of their HF state-dict key, each as rng.standard_normal(shape) * std
  (float64 -> float32) with
    * linear / conv weights and biases          std lin_std (default 0.02)
    * decoder.embed_tokens                      std 0.25 (peaky softmax)
    * decoder.embed_positions                   std 0.02
    * LayerNorm weight = 1 + 0.1 * N(0,1),  bias = 0.02 * N(0,1)
  encoder.embed_positions is the sinusoid table (HF:modeling_whisper.py:55-64),
  which is what real checkpoints carry.
"""
from __future__ import annotations

import math

import numpy as np

SPECIAL = dict(
    eot=50257, pad=50257, sot=50258, en=50259, zh=50260, transcribe=50359,
    translate=50358, startofprev=50361, nospeech=50362, notimestamps=50363,
    timestamp_begin=50364,
)


def _base(d, el, dl, h, ffn, vocab=51865, max_src=1500, max_tgt=448):
    return dict(
        d_model=d, encoder_layers=el, decoder_layers=dl,
        encoder_attention_heads=h, decoder_attention_heads=h,
        encoder_ffn_dim=ffn, decoder_ffn_dim=ffn, vocab_size=vocab,
        num_mel_bins=80, max_source_positions=max_src, max_target_positions=max_tgt,
        pad_token_id=SPECIAL["pad"], bos_token_id=SPECIAL["eot"], eos_token_id=SPECIAL["eot"],
        decoder_start_token_id=SPECIAL["sot"], activation_function="gelu",
        scale_embedding=False, dropout=0.0, attention_dropout=0.0, activation_dropout=0.0,
        layerdrop=0.0, encoder_layerdrop=0.0, decoder_layerdrop=0.0,
        tie_word_embeddings=True,
    )


CONFIGS = {
    # micro: parity-test config (full vocab, real mel/encoder lengths)
    "micro": _base(128, 2, 2, 2, 256),
    "tiny": _base(384, 4, 4, 6, 1536),
    "base": _base(512, 6, 6, 8, 2048),
    "small": _base(768, 12, 12, 12, 3072),
    "medium": _base(1024, 24, 24, 16, 4096),
    "large-v2": _base(1280, 32, 32, 20, 5120),
    "distil-32-2": _base(1280, 32, 2, 20, 5120),
}


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """HF:modeling_whisper.py:55-64 (computed in float32 like torch)."""
    import torch

    log_inc = math.log(max_timescale) / (channels // 2 - 1)
    inv = torch.exp(-log_inc * torch.arange(channels // 2))
    t = torch.arange(length).view(-1, 1) * inv.view(1, -1)
    return torch.cat([t.sin(), t.cos()], dim=1).numpy().astype(np.float32)


def param_shapes(cfg: dict) -> dict:
    """HF state-dict key -> shape (WhisperForConditionalGeneration, proj_out tied)."""
    d, V = cfg["d_model"], cfg["vocab_size"]
    s = {}
    s["model.encoder.conv1.weight"] = (d, cfg["num_mel_bins"], 3)
    s["model.encoder.conv1.bias"] = (d,)
    s["model.encoder.conv2.weight"] = (d, d, 3)
    s["model.encoder.conv2.bias"] = (d,)
    s["model.encoder.embed_positions.weight"] = (cfg["max_source_positions"], d)

    def attn(p):
        s[p + ".q_proj.weight"] = (d, d); s[p + ".q_proj.bias"] = (d,)
        s[p + ".k_proj.weight"] = (d, d)
        s[p + ".v_proj.weight"] = (d, d); s[p + ".v_proj.bias"] = (d,)
        s[p + ".out_proj.weight"] = (d, d); s[p + ".out_proj.bias"] = (d,)

    def ln(p):
        s[p + ".weight"] = (d,); s[p + ".bias"] = (d,)

    def mlp(p, f):
        s[p + ".fc1.weight"] = (f, d); s[p + ".fc1.bias"] = (f,)
        s[p + ".fc2.weight"] = (d, f); s[p + ".fc2.bias"] = (d,)

    for i in range(cfg["encoder_layers"]):
        p = f"model.encoder.layers.{i}"
        attn(p + ".self_attn"); ln(p + ".self_attn_layer_norm")
        mlp(p, cfg["encoder_ffn_dim"]); ln(p + ".final_layer_norm")
    ln("model.encoder.layer_norm")
    s["model.decoder.embed_tokens.weight"] = (V, d)
    s["model.decoder.embed_positions.weight"] = (cfg["max_target_positions"], d)
    for i in range(cfg["decoder_layers"]):
        p = f"model.decoder.layers.{i}"
        attn(p + ".self_attn"); ln(p + ".self_attn_layer_norm")
        attn(p + ".encoder_attn"); ln(p + ".encoder_attn_layer_norm")
        mlp(p, cfg["decoder_ffn_dim"]); ln(p + ".final_layer_norm")
    ln("model.decoder.layer_norm")
    return s


def _scale(k, z, lin_std, embed_std=0.25):
    if "layer_norm" in k:
        w = 1.0 + 0.1 * z if k.endswith("weight") else 0.02 * z
    elif k.endswith("embed_tokens.weight"):
        w = embed_std * z
    elif k.endswith("embed_positions.weight"):
        w = 0.02 * z
    else:
        w = lin_std * z
    return w.astype(np.float32)


def make_weights(cfg: dict, seed: int, lin_std: float = 0.02, per_tensor: bool = False, embed_std: float = 0.25) -> dict:
    """Deterministic HF-keyed float32 state dict (numpy). proj_out is tied, not listed.

    per_tensor=False: one PCG64(seed) stream over the sorted keys (the micro / tiny fixtures).
    per_tensor=True (the BASELINE-size fixtures, large-v2 has 1.5 G weights): tensor i of the sorted
    keys draws from its own PCG64([seed, i]) stream, so the tensors are generated in parallel
    threads (numpy releases the GIL while filling) with the same values on any machine.
    embed_std: std of decoder.embed_tokens (0.25 makes the micro config's softmax peaky; at real widths
    it makes every position predict its own input token, so the BASELINE-size fixtures use 0.05)."""
    shapes = param_shapes(cfg)
    keys = sorted(shapes)
    if not per_tensor:
        rng = np.random.Generator(np.random.PCG64(seed))
        out = {}
        for k in keys:
            z = rng.standard_normal(shapes[k])
            out[k] = sinusoids(*shapes[k]) if k.endswith("encoder.embed_positions.weight") else \
                _scale(k, z, lin_std, embed_std)
        return out
    from concurrent.futures import ThreadPoolExecutor

    def one(i):
        k = keys[i]
        if k.endswith("encoder.embed_positions.weight"):
            return k, sinusoids(*shapes[k])
        z = np.random.Generator(np.random.PCG64([seed, i])).standard_normal(shapes[k])
        return k, _scale(k, z, lin_std, embed_std)
    with ThreadPoolExecutor(max_workers=min(16, len(keys))) as ex:
        return dict(ex.map(one, range(len(keys))))
