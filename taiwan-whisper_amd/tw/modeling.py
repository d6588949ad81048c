"""MI355X-native Whisper encoder-decoder (drop-in for the parts of HF
`WhisperForConditionalGeneration` the taiwan-whisper distillation path touches).

Reference contract: `from_pretrained(dir, torch_dtype=...)`,
`model(input_features, decoder_input_ids, labels) -> .loss/.logits/.encoder_last_hidden_state`,
`model(encoder_outputs=..., labels=...)` with shift_tokens_right semantics
(`training/run_distillation.py:1528-1537`), `.save_pretrained`, HF state-dict key names,
`.model.encoder/.model.decoder` parameter groups for freezing (`:1043-1066`).

Engine layout (MI355X-first):
  * every parameter lives in ONE flat buffer (fp32 master `p32` for trainable models,
    always a bf16 mirror `p16` — the autocast weight cast done once per update, by the
    AdamW kernel, instead of once per forward);
  * q/k/v (and cross-attn k/v) are adjacent so the fused QKV / KV projection weight is a
    view; the missing k_proj bias is a zero segment;
  * conv weights are stored [d][tap][c] so the conv stem is two batched GEMMs over
    zero-copy strided views of the time-major input (no im2col in the forward);
  * embed_tokens is padded to a multiple of 64 rows (51865 -> 51904) with zero rows, so
    logits / dlogits rows are 16-B aligned and every GEMM dim is MFMA-friendly.
Arithmetic follows CUDA bf16 autocast (ACC:accelerator.py:1818-1829) exactly as
oracle/whisper_ref.py restates it; every matmul / norm / softmax runs in libtw_hip.so.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import ops
from .config import GenerationConfig, WhisperConfig

_DEFER_RES = os.environ.get("TW_DEFER_RES", "1")   # "0": never, "2": fp32 streams only, else default
_LN_G16 = os.environ.get("TW_LN_G16", "1") != "0"  # "0": the backward casts the stream gradient separately (A/B runs)

F = ops


def padded_vocab(V: int) -> int:
    return (V + 63) // 64 * 64



def fp32_compute_supported() -> bool:
    """The fp32-arithmetic path (mixed_precision="no": tw_gemm_f32 / tw_attn_*_f32 and the fp32 variants of
    the loss, decode and selection kernels) is part of libtw_hip.so."""
    return True

# ---------------------------------------------------------------------------------------------
# parameter layout
def _attn_segs(p, d, fused_kv_only=False):
    segs = []
    if not fused_kv_only:
        segs += [(p + ".q_proj.weight", (d, d)), (p + ".k_proj.weight", (d, d)), (p + ".v_proj.weight", (d, d)),
                 (p + ".q_proj.bias", (d,)), (p + ".k_proj.zero_bias", (d,)), (p + ".v_proj.bias", (d,))]
    else:  # cross attention: q separate, k/v fused
        segs += [(p + ".q_proj.weight", (d, d)), (p + ".q_proj.bias", (d,)),
                 (p + ".k_proj.weight", (d, d)), (p + ".v_proj.weight", (d, d)),
                 (p + ".k_proj.zero_bias", (d,)), (p + ".v_proj.bias", (d,))]
    segs += [(p + ".out_proj.weight", (d, d)), (p + ".out_proj.bias", (d,))]
    return segs


def engine_segments(cfg: WhisperConfig):
    """Ordered (name, engine_shape) list.  Names are HF state-dict keys (plus the
    non-parameter `*.k_proj.zero_bias` segments)."""
    d, Vp = cfg.d_model, padded_vocab(cfg.vocab_size)
    segs = [("model.encoder.conv1.weight", (d, 3 * cfg.num_mel_bins)), ("model.encoder.conv1.bias", (d,)),
            ("model.encoder.conv2.weight", (d, 3 * d)), ("model.encoder.conv2.bias", (d,)),
            ("model.encoder.embed_positions.weight", (cfg.max_source_positions, d))]

    def ln(p):
        return [(p + ".weight", (d,)), (p + ".bias", (d,))]

    def mlp(p, f):
        return [(p + ".fc1.weight", (f, d)), (p + ".fc1.bias", (f,)), (p + ".fc2.weight", (d, f)),
                (p + ".fc2.bias", (d,))]

    for i in range(cfg.encoder_layers):
        p = f"model.encoder.layers.{i}"
        segs += ln(p + ".self_attn_layer_norm") + _attn_segs(p + ".self_attn", d)
        segs += ln(p + ".final_layer_norm") + mlp(p, cfg.encoder_ffn_dim)
    segs += ln("model.encoder.layer_norm")
    segs += [("model.decoder.embed_tokens.weight", (Vp, d)),
             ("model.decoder.embed_positions.weight", (cfg.max_target_positions, d))]
    for i in range(cfg.decoder_layers):
        p = f"model.decoder.layers.{i}"
        segs += ln(p + ".self_attn_layer_norm") + _attn_segs(p + ".self_attn", d)
        segs += ln(p + ".encoder_attn_layer_norm") + _attn_segs(p + ".encoder_attn", d, fused_kv_only=True)
        segs += ln(p + ".final_layer_norm") + mlp(p, cfg.decoder_ffn_dim)
    segs += ln("model.decoder.layer_norm")
    return segs


def is_pseudo(name):
    return name.endswith(".zero_bias")


def to_engine(name, t: torch.Tensor, cfg: WhisperConfig, eng_shape):
    """HF tensor -> engine layout (host)."""
    if name.endswith("conv1.weight") or name.endswith("conv2.weight"):
        return t.permute(0, 2, 1).reshape(eng_shape)          # [d][c][k] -> [d][k][c]
    if name.endswith("embed_tokens.weight"):
        out = torch.zeros(eng_shape, dtype=t.dtype)
        out[: t.shape[0]] = t
        return out
    return t.reshape(eng_shape)


def to_hf(name, v: torch.Tensor, cfg: WhisperConfig):
    """engine view -> HF-shaped view (no copy)."""
    if name.endswith("conv1.weight") or name.endswith("conv2.weight"):
        d, kc = v.shape
        return v.view(d, 3, kc // 3).permute(0, 2, 1)
    if name.endswith("embed_tokens.weight"):
        return v[: cfg.vocab_size]
    return v


class ParamStore:
    """Flat device buffers with named engine-layout views."""

    def __init__(self, segs, device, master: bool, order=None, half=torch.bfloat16):
        self.segs = dict(segs)
        names = [n for n, _ in segs] if order is None else list(order)
        self.order = names
        self.offset, off = {}, 0
        for n in names:
            self.offset[n] = off
            off += int(np.prod(self.segs[n]))
            off = (off + 63) // 64 * 64
        self.total = off
        self.device = device
        self.p32 = torch.zeros(off, dtype=torch.float32, device=device) if master else None
        # the 16-bit copy the GEMMs read: the bf16 mirror (autocast's weight cast), or the fp16 weights of a
        # torch_dtype=float16 model
        self.p16 = torch.zeros(off, dtype=half, device=device)

    def numel(self, n):
        return int(np.prod(self.segs[n]))

    def _view(self, buf, n):
        o = self.offset[n]
        return buf[o: o + self.numel(n)].view(self.segs[n])

    def v32(self, n):
        return self._view(self.p32, n)

    def v16(self, n):
        return self._view(self.p16, n)

    def span(self, buf, first, last, shape):
        o0, o1 = self.offset[first], self.offset[last] + self.numel(last)
        assert o1 - o0 == int(np.prod(shape)), (first, last)
        return buf[o0:o1].view(shape)


@dataclass
class Seq2SeqOutput:
    loss: Optional[torch.Tensor] = None
    logits: Optional[torch.Tensor] = None               # [B, T, V] view of the padded bf16 logits
    encoder_last_hidden_state: Optional[torch.Tensor] = None   # [B, 1500, d] bf16
    logits_padded: Optional[torch.Tensor] = None        # [B*T, Vp] bf16


@dataclass
class BaseModelOutput:
    last_hidden_state: torch.Tensor


class _Group:
    """Parameter-group shim for `model.model.encoder` etc. (freezing, counting)."""

    def __init__(self, model, prefix):
        self._m, self._p = model, prefix

    def named_parameters(self):
        for n, v in self._m.named_parameters():
            if n.startswith(self._p):
                yield n, v

    def parameters(self):
        return (v for _, v in self.named_parameters())

    def requires_grad_(self, flag=True):
        self._m.set_trainable(self._p, flag)
        return self

    def __getattr__(self, item):
        sub = self._p + "." + item
        if item == "layers":
            n = self._m.config.encoder_layers if self._p.endswith("encoder") else self._m.config.decoder_layers
            return [_Group(self._m, f"{sub}.{i}") for i in range(n)]
        return _Group(self._m, sub)

    @property
    def weight(self):
        return self._m.state_view(self._p + ".weight")


class WhisperForConditionalGeneration:
    main_input_name = "input_features"

    def __init__(self, config: WhisperConfig, dtype=torch.float32, device="cuda", compute: str = "bf16"):
        """dtype: parameter storage (fp32 master + bf16 mirror, bf16 only, or fp16 only).  compute: "bf16" = CUDA
        bf16 autocast's rounding points (mixed_precision="bf16", every reference launcher); "fp32" = plain fp32
        arithmetic end to end (mixed_precision="no", the reference's default --dtype float32; needs the
        fp32 master); "fp16" = a torch_dtype=float16 model without autocast (run_eval.py:99,500-509 default
        --dtype float16, run_pseudo_labelling.py:461-463): fp16 weights, fp16 Linear / attention outputs and
        residual stream, LayerNorm statistics in fp32 with fp16 output, fp16 logits -- inference and the fp16
        teacher of fp16 distillation; on an fp32-master model "fp16" is CUDA fp16 AUTOCAST (mixed_precision="fp16",
        run_distillation.py:815-817): the bf16 path's rounding points with fp16 in place of bf16 (fp32 stream)."""
        if isinstance(config, dict):
            config = WhisperConfig(**config)
        self.config = config
        self.dtype = dtype
        self.compute = "bf16"
        self.device = torch.device(device)
        self.Vp = padded_vocab(config.vocab_size)
        self.segs = engine_segments(config)
        if dtype not in (torch.float32, torch.bfloat16, torch.float16):
            raise ValueError(f"unsupported parameter dtype {dtype}")
        self.store = ParamStore(self.segs, self.device, master=(dtype == torch.float32),
                                half=torch.float16 if (dtype == torch.float16 or compute == "fp16") else torch.bfloat16)
        self._ln32 = {}          # fp32 LayerNorm params for bf16 models
        self.trainable = set()   # HF names with requires_grad
        self.grad = None         # flat fp32 grads over the trainable prefix (see pack_for_training)
        self.train_prefix = 0
        self.generation_config = None
        self.training = False
        self.model = _Group(self, "model")
        self.model.encoder = _Group(self, "model.encoder")
        self.model.decoder = _Group(self, "model.decoder")
        self.proj_out = _Group(self, "model.decoder.embed_tokens")
        self.set_compute("fp16" if dtype == torch.float16 else compute)

    def set_compute(self, compute: str):
        if compute not in ("bf16", "fp32", "fp16"):
            raise ValueError(f"compute must be 'bf16', 'fp16' or 'fp32', got {compute!r}")
        if compute == "fp32" and self.dtype != torch.float32:
            raise ValueError("fp32 arithmetic needs fp32 parameters (torch_dtype=torch.float32)")
        if self.dtype == torch.float16 and compute != "fp16":
            raise ValueError("a torch_dtype=float16 model computes in fp16 only")
        if self.dtype == torch.bfloat16 and compute == "fp16":
            raise ValueError("fp16 arithmetic needs fp16 parameters or an fp32 master (fp16 autocast)")
        self.compute = compute
        # fp32-master model: the 16-bit mirror is autocast's weight cast, in the autocast dtype
        half = torch.float16 if compute == "fp16" else torch.bfloat16
        if self.store.p32 is not None and compute != "fp32" and self.store.p16.dtype != half:
            self.store.p16 = torch.empty(self.store.total, dtype=half, device=self.device)
            F.cast_bf16(self.store.p32, self.store.p16)
        return self

    @property
    def act_dtype(self):
        """dtype of every GEMM / attention operand and output: bf16 under autocast, fp32 on the fp32 path, fp16 for
        an fp16 model."""
        return {"fp32": torch.float32, "fp16": torch.float16}.get(self.compute, torch.bfloat16)

    def act_grad(self, g: torch.Tensor) -> torch.Tensor:
        """gradient entering a GEMM: rounded to the autocast dtype (the grad of a bf16 / fp16 activation),
        unchanged on the fp32 path."""
        return g if self.compute == "fp32" else _half(g, self.act_dtype)

    # ------------------------------------------------------------------ state dict / IO
    @property
    def stream_dtype(self):
        return self.dtype

    def named_parameters(self):
        for n in self.store.order:
            if not is_pseudo(n):
                yield n, self.state_view(n)

    def parameters(self):
        return (v for _, v in self.named_parameters())

    def num_parameters(self, only_trainable=False):
        return sum(self.config_numel(n) for n in self.store.order
                   if not is_pseudo(n) and (not only_trainable or n in self.trainable))

    def config_numel(self, n):
        if n.endswith("embed_tokens.weight"):
            return self.config.vocab_size * self.config.d_model
        return self.store.numel(n)

    def state_view(self, n):
        buf = self.store.p32 if self.store.p32 is not None else self.store.p16
        return to_hf(n, self.store._view(buf, n), self.config)

    def state_dict(self):
        sd = {n: self.state_view(n) for n in self.store.order if not is_pseudo(n)}
        sd["proj_out.weight"] = sd["model.decoder.embed_tokens.weight"]
        return sd

    def load_state_dict(self, sd: dict, strict=True):
        missing = []
        for n, shp in self.segs:
            if is_pseudo(n):
                continue
            if n not in sd:
                missing.append(n)
                continue
            t = torch.as_tensor(sd[n])
            eng = to_engine(n, t, self.config, shp)
            if self.store.p32 is not None:
                self.store.v32(n).copy_(eng.to(torch.float32))
            self.store.v16(n).copy_(eng.to(self.store.p16.dtype))
        unexpected = [k for k in sd if k not in self.store.segs and k != "proj_out.weight"]
        if strict and (missing or unexpected):
            raise RuntimeError(f"load_state_dict: missing {missing[:5]} unexpected {unexpected[:5]}")
        self._refresh_ln32()
        return missing, unexpected

    def _refresh_ln32(self):
        self._ln32 = {}
        if self.store.p32 is None:
            for n in self.store.order:
                if "layer_norm" in n:
                    self._ln32[n] = self.store.v16(n).float()

    def ln_param(self, n):
        return self.store.v32(n) if self.store.p32 is not None else self._ln32[n]

    @classmethod
    def from_state_dict(cls, config, sd, dtype=torch.float32, device="cuda", compute="bf16"):
        m = cls(config, dtype=dtype, device=device, compute=compute)
        m.load_state_dict(sd, strict=False)
        return m

    @classmethod
    def from_pretrained(cls, path, torch_dtype=None, attn_implementation=None, low_cpu_mem_usage=True, config=None,
                        device="cuda", compute="bf16", **kw):
        from safetensors.torch import load_file
        cfg = config if config is not None else WhisperConfig.from_pretrained(path)
        if isinstance(cfg, dict):
            cfg = WhisperConfig(**cfg)
        sd = load_file(os.path.join(path, "model.safetensors"))
        dt = torch_dtype or torch.float32
        m = cls.from_state_dict(cfg, sd, dtype=dt, device=device, compute="fp16" if dt == torch.float16 else compute)
        gp = os.path.join(path, "generation_config.json")
        if os.path.exists(gp):
            with open(gp) as f:
                m.generation_config = GenerationConfig(json.load(f))
        return m

    def save_pretrained(self, path):
        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        self.config.save_pretrained(path)
        sd = {n: v.detach().to("cpu").contiguous() for n, v in self.state_dict().items() if n != "proj_out.weight"}
        save_file(sd, os.path.join(path, "model.safetensors"), metadata={"format": "pt"})
        if self.generation_config is not None:
            with open(os.path.join(path, "generation_config.json"), "w") as f:
                json.dump(dict(self.generation_config), f, indent=2)

    # ------------------------------------------------------------------ training layout
    def set_trainable(self, prefix, flag):
        for n in self.store.order:
            if n.startswith(prefix) and not is_pseudo(n):
                if flag:
                    self.trainable.add(n)
                else:
                    self.trainable.discard(n)

    def gradient_checkpointing_enable(self, **kw):
        """Accepted for API parity; activations are kept in HBM (288 GB) instead of recomputed."""
        self.gradient_checkpointing = True

    def train(self, mode=True):
        self.training = mode
        return self

    def eval(self):
        return self.train(False)

    def pack_for_training(self):
        """Re-lay the flat buffers as [trainable (module order) | frozen] and allocate the flat
        fp32 gradient over the trainable prefix (one AdamW / norm / all-reduce range)."""
        assert self.store.p32 is not None, "only fp32-master models are trained"
        names = [n for n, _ in self.segs]
        if "model.decoder.embed_positions.weight" in self.trainable:
            pass
        owner = lambda n: n.replace(".k_proj.zero_bias", ".q_proj.bias")
        tr = [n for n in names if (owner(n) in self.trainable)]
        fr = [n for n in names if owner(n) not in self.trainable]
        old = self.store
        new = ParamStore(self.segs, self.device, master=True, order=tr + fr, half=old.p16.dtype)
        for n in names:
            new.v32(n).copy_(old.v32(n))
            new.v16(n).copy_(old.v16(n))
        self.store = new
        self.train_names = tr
        self.train_prefix = new.offset[tr[-1]] + new.numel(tr[-1]) if tr else 0
        self.train_prefix = (self.train_prefix + 63) // 64 * 64
        self.grad = torch.zeros(self.train_prefix, dtype=torch.float32, device=self.device)
        return self

    def gv(self, n):
        """flat-gradient view of a trainable segment (engine layout) or None if frozen."""
        if self.grad is None or n not in self.trainable and not is_pseudo(n):
            return None
        o = self.store.offset[n]
        if o >= self.train_prefix:
            return None
        return self.grad[o: o + self.store.numel(n)].view(self.store.segs[n])

    def grad_range(self, prefix):
        """(lo, hi) of the flat-gradient slice holding every trainable segment named prefix*, or None."""
        lo, hi = None, None
        for n in self.store.order:
            if not n.startswith(prefix):
                continue
            o = self.store.offset[n]
            if o >= self.train_prefix:
                continue
            e = o + self.store.numel(n)
            lo = o if lo is None else min(lo, o)
            hi = e if hi is None else max(hi, e)
        return None if lo is None else (lo, hi)

    def sync_bf16(self):
        """16-bit mirror := bf16 / fp16 (fp32 master) (autocast's weight cast) for the whole model."""
        if self.store.p32 is not None:
            F.cast_bf16(self.store.p32, self.store.p16)

    # ------------------------------------------------------------------ building blocks
    def _w16(self, n):
        """weight as the GEMMs read it: the bf16 mirror (autocast's weight cast), or the fp32 master on
        the fp32 path."""
        return self.store.v32(n) if self.compute == "fp32" else self.store.v16(n)

    def wspan(self, first, last, shape):
        """fused projection weight / bias spanning adjacent segments (compute dtype)."""
        buf = self.store.p32 if self.compute == "fp32" else self.store.p16
        return self.store.span(buf, first, last, shape)

    def _lin(self, x, w, b, out, flags=F.GEMM_ROUND, res=None, aux=None, M=None):
        M = x.shape[0] if M is None else M
        N, K = w.shape
        F.gemm(x, w, out, M, N, K, lda=x.stride(0), ldb=K, ldc=out.stride(0), bias=b, res=res,
               ldr=res.stride(0) if res is not None else 0, aux=aux, ldaux=aux.stride(0) if aux is not None else 0,
               flags=flags)
        return out

    def _ln(self, x, name, out_dtype=None, save=None):
        y = torch.empty(x.shape, dtype=out_dtype or self.act_dtype, device=self.device)
        mean = rstd = None
        if save is not None:
            mean = torch.empty(x.shape[0], dtype=torch.float32, device=self.device)
            rstd = torch.empty_like(mean)
            save[name] = (x, mean, rstd, y)
        F.layernorm_fwd(x, self.ln_param(name + ".weight"), self.ln_param(name + ".bias"), y, mean, rstd)
        return y

    def defer_residual(self, kind):
        """Whether the stream-updating Linear of a `kind` block ("attn" = out_proj, "mlp" = fc2) writes its bf16
        output and leaves the residual add to the next LayerNorm (tw_add_layernorm_fwd, the same add): on the
        student's fp32 stream for both (the fp32 read-modify-write leaves the persistent GEMM's epilogue), on
        the bf16 teacher stream for out_proj only (the plain-bias projection then runs the store-only epilogue; at
        fc2 the extra LN traffic costs what the epilogue saves).  DESIGN.md §5; TW_DEFER_RES=0 disables (A/B runs)."""
        # tw_add_layernorm_fwd: D % 256 == 0 and D <= 1280 (every Whisper size), else the residual epilogue
        if _DEFER_RES == "0" or self.act_dtype == torch.float32 or self.config.d_model % 256 or self.config.d_model > 1280:
            return False
        if self.act_dtype == torch.float16:
            # fp16 autocast's fp32 stream (tw_add_layernorm_fwd_f16); the fp16 model's fp16 stream keeps the residual
            # epilogue, which also applies the encoder's fp16 clamp
            return self.stream_dtype == torch.float32
        return self.stream_dtype == torch.float32 or (kind == "attn" and _DEFER_RES != "2")

    def _ln_in(self, x, pend, name, save):
        """Block-entry LayerNorm -> (stream, LN output).  pend: a deferred residual update (bf16), added to
        the stream first (in place, or into a fresh buffer when a tape holds the old stream)."""
        if pend is None:
            return x, self._ln(x, name, save=save)
        xn = x if save is None else torch.empty_like(x)
        y = torch.empty(x.shape, dtype=self.act_dtype, device=self.device)
        mean = rstd = None
        if save is not None:
            mean = torch.empty(x.shape[0], dtype=torch.float32, device=self.device)
            rstd = torch.empty_like(mean)
            save[name] = (xn, mean, rstd, y)
        F.add_layernorm_fwd(x, pend, xn, self.ln_param(name + ".weight"), self.ln_param(name + ".bias"), y, mean, rstd)
        return xn, y

    def _res_out(self, h, w, b, x, tape, kind, clamp=False):
        """The stream-updating Linear -> (stream, pending update): deferred to the next LayerNorm
        (defer_residual), else applied by the GEMM's residual epilogue.  clamp: the fp16 encoder layer's
        saturation after its MLP residual (HF modeling_whisper.py:409-411), fused into that epilogue."""
        M, N = h.shape[0], w.shape[0]
        if self.defer_residual(kind):
            r = torch.empty(M, N, dtype=self.act_dtype, device=self.device)
            self._lin(h, w, b, r)
            return x, r
        out = torch.empty(M, N, dtype=self.stream_dtype, device=self.device) if tape is not None else x
        # HF clamps only an fp16 STREAM (modeling_whisper.py:409-411): the fp16 model's, not fp16 autocast's fp32 one
        flags = F.GEMM_ROUND | (F.GEMM_CLAMP16 if clamp and self.stream_dtype == torch.float16 else 0)
        self._lin(h, w, b, out, res=x, flags=flags)
        return out, None

    def _attn_block(self, x, p, B, T, causal, tape=None, pend=None):
        """x: residual stream [B*T, d] (+ a pending update) -> (new stream, pending update) (self attention)."""
        cfg, d = self.config, self.config.d_model
        H = d // 64
        sv = {} if tape is not None else None
        x, y = self._ln_in(x, pend, p + "_layer_norm", sv)
        M = B * T
        qkv = torch.empty(M, 3 * d, dtype=self.act_dtype, device=self.device)
        wqkv = self.wspan(p + ".q_proj.weight", p + ".v_proj.weight", (3 * d, d))
        bqkv = self.wspan(p + ".q_proj.bias", p + ".v_proj.bias", (3 * d,))
        self._lin(y, wqkv, bqkv, qkv)
        o = torch.empty(M, d, dtype=self.act_dtype, device=self.device)
        lse = torch.empty(B * H * T, dtype=torch.float32, device=self.device) if tape is not None else None
        F.attn_fwd(qkv, 3 * d, qkv[:, d:], 3 * d, qkv[:, 2 * d:], 3 * d, o, d, lse, B, H, T, T, causal, 0.125)
        out = self._res_out(o, self._w16(p + ".out_proj.weight"), self._w16(p + ".out_proj.bias"), x, tape, "attn")
        if tape is not None:
            tape.append(("attn", p, dict(sv=sv, y=y, qkv=qkv, o=o, lse=lse, B=B, T=T, causal=causal)))
        return out

    def _cross_block(self, x, enc16, p, B, T, Tk, tape=None, kv=None, pend=None):
        d = self.config.d_model
        H = d // 64
        sv = {} if tape is not None else None
        x, y = self._ln_in(x, pend, p + "_layer_norm", sv)
        M = B * T
        q = torch.empty(M, d, dtype=self.act_dtype, device=self.device)
        self._lin(y, self._w16(p + ".q_proj.weight"), self._w16(p + ".q_proj.bias"), q)
        if kv is None:
            kv = torch.empty(B * Tk, 2 * d, dtype=self.act_dtype, device=self.device)
            wkv = self.wspan(p + ".k_proj.weight", p + ".v_proj.weight", (2 * d, d))
            bkv = self.wspan(p + ".k_proj.zero_bias", p + ".v_proj.bias", (2 * d,))
            self._lin(enc16, wkv, bkv, kv)
        o = torch.empty(M, d, dtype=self.act_dtype, device=self.device)
        lse = torch.empty(B * H * T, dtype=torch.float32, device=self.device) if tape is not None else None
        F.attn_fwd(q, d, kv, 2 * d, kv[:, d:], 2 * d, o, d, lse, B, H, T, Tk, False, 0.125)
        out = self._res_out(o, self._w16(p + ".out_proj.weight"), self._w16(p + ".out_proj.bias"), x, tape, "attn")
        if tape is not None:
            tape.append(("cross", p, dict(sv=sv, y=y, q=q, kv=kv, o=o, lse=lse, B=B, T=T, Tk=Tk)))
        return out

    def _mlp_block(self, x, p, tape=None, pend=None, clamp=False):
        M = x.shape[0]
        sv = {} if tape is not None else None
        x, y = self._ln_in(x, pend, p + ".final_layer_norm", sv)
        f = self.store.segs[p + ".fc1.weight"][0]
        h = torch.empty(M, f, dtype=self.act_dtype, device=self.device)
        pre = torch.empty(M, f, dtype=self.act_dtype, device=self.device) if tape is not None else None
        self._lin(y, self._w16(p + ".fc1.weight"), self._w16(p + ".fc1.bias"), h, aux=pre,
                  flags=F.GEMM_ROUND | F.GEMM_GELU | (F.GEMM_AUX_OUT if tape is not None else 0))
        out = self._res_out(h, self._w16(p + ".fc2.weight"), self._w16(p + ".fc2.bias"), x, tape, "mlp", clamp=clamp)
        if tape is not None:
            tape.append(("mlp", p, dict(sv=sv, y=y, h=h, pre=pre)))
        return out

    # ------------------------------------------------------------------ encoder / decoder
    def conv_input(self, input_features: torch.Tensor) -> torch.Tensor:
        """[B, 80, 3000] fp32 -> time-major padded [B, 3002, 80] in the compute dtype (the log-mel kernel
        emits the bf16 one directly; this path serves callers that hand over input_features)."""
        B, nm, T = input_features.shape
        if T != 2 * self.config.max_source_positions:
            raise ValueError(f"Whisper expects the mel input features to be of length "
                             f"{2 * self.config.max_source_positions}, but found {T}.")
        xt = torch.empty(B, T + 2, nm, dtype=self.act_dtype, device=self.device)
        F.mel_to_conv_input(input_features.to(self.device, torch.float32).contiguous(), xt)
        return xt

    def encode(self, conv_in: torch.Tensor, tape=None) -> torch.Tensor:
        """conv_in [B, 3002, 80] -> encoder_last_hidden_state [B*1500, d] (compute dtype)."""
        cfg, d = self.config, self.config.d_model
        B, T2 = conv_in.shape[0], conv_in.shape[1] - 2
        T = T2 // 2
        nm = cfg.num_mel_bins
        if conv_in.dtype != self.act_dtype:
            raise ValueError(f"conv input is {conv_in.dtype}, this model computes in {self.act_dtype}")
        H1 = torch.empty(B, T2 + 2, d, dtype=self.act_dtype, device=self.device)
        H1[:, 0].zero_()
        H1[:, T2 + 1].zero_()
        pre1 = pre2 = None
        if tape is not None:
            pre1 = torch.empty(B, T2, d, dtype=self.act_dtype, device=self.device)
            pre2 = torch.empty(B, T, d, dtype=self.act_dtype, device=self.device)
        gf = F.GEMM_ROUND | F.GEMM_GELU | (F.GEMM_AUX_OUT if tape is not None else 0)
        F.gemm(conv_in, self._w16("model.encoder.conv1.weight"), H1[:, 1:], T2, d, 3 * nm, lda=nm, ldb=3 * nm,
               ldc=d, batch=B, sA=(T2 + 2) * nm, sC=(T2 + 2) * d, bias=self._w16("model.encoder.conv1.bias"),
               aux=pre1, ldaux=d, sAux=T2 * d, flags=gf)
        x = torch.empty(B * T, d, dtype=self.stream_dtype, device=self.device)
        pos = self.store.v32("model.encoder.embed_positions.weight") if self.store.p32 is not None \
            else self.store.v16("model.encoder.embed_positions.weight")
        F.gemm(H1, self._w16("model.encoder.conv2.weight"), x, T, d, 3 * d, lda=2 * d, ldb=3 * d, ldc=d, batch=B,
               sA=(T2 + 2) * d, sC=T * d, bias=self._w16("model.encoder.conv2.bias"), res=pos, ldr=d, res_mod=T,
               aux=pre2, ldaux=d, sAux=T * d, flags=gf)
        if tape is not None:
            tape.append(("conv", "model.encoder", dict(conv_in=conv_in, H1=H1, pre1=pre1, pre2=pre2, B=B, T=T)))
        pend = None
        for i in range(cfg.encoder_layers):
            p = f"model.encoder.layers.{i}"
            x, pend = self._attn_block(x, p + ".self_attn", B, T, False, tape, pend)
            x, pend = self._mlp_block(x, p, tape, pend, clamp=True)
        sv = {} if tape is not None else None
        _, enc = self._ln_in(x, pend, "model.encoder.layer_norm", sv)
        if tape is not None:
            tape.append(("ln_final", "model.encoder.layer_norm", dict(sv=sv)))
        return enc

    def embed(self, ids: torch.Tensor) -> torch.Tensor:
        B, T = ids.shape
        d = self.config.d_model
        if self.store.p32 is not None:
            tok, pos = self.store.v32("model.decoder.embed_tokens.weight"), self.store.v32(
                "model.decoder.embed_positions.weight")
        else:
            tok, pos = self.store.v16("model.decoder.embed_tokens.weight"), self.store.v16(
                "model.decoder.embed_positions.weight")
        x = torch.empty(B * T, d, dtype=self.stream_dtype, device=self.device)
        F.embed_fwd(ids.reshape(-1).contiguous(), tok, pos, x, T)
        return x

    def decode(self, ids: torch.Tensor, enc16: torch.Tensor, Tk: int, tape=None) -> torch.Tensor:
        """ids [B, T] int64 (device), enc16 [B*Tk, d] -> final decoder hidden [B*T, d] (compute dtype)."""
        cfg = self.config
        B, T = ids.shape
        if T > cfg.max_target_positions:
            raise ValueError("decoder input longer than max_target_positions")
        x = self.embed(ids)
        if tape is not None:
            tape.append(("embed", "model.decoder", dict(ids=ids.reshape(-1).contiguous(), B=B, T=T)))
        pend = None
        for i in range(cfg.decoder_layers):
            p = f"model.decoder.layers.{i}"
            x, pend = self._attn_block(x, p + ".self_attn", B, T, True, tape, pend)
            x, pend = self._cross_block(x, enc16, p + ".encoder_attn", B, T, Tk, tape, pend=pend)
            x, pend = self._mlp_block(x, p, tape, pend)
        sv = {} if tape is not None else None
        _, h = self._ln_in(x, pend, "model.decoder.layer_norm", sv)
        if tape is not None:
            tape.append(("ln_final", "model.decoder.layer_norm", dict(sv=sv)))
        return h

    def lm_head(self, h16: torch.Tensor, out=None) -> torch.Tensor:
        """tied proj_out: [M, d] -> logits [M, Vp] in the compute dtype (pad columns are 0)."""
        M = h16.shape[0]
        if out is None:
            out = torch.empty(M, self.Vp, dtype=self.act_dtype, device=self.device)
        E = self._w16("model.decoder.embed_tokens.weight")
        F.gemm(h16, E, out, M, self.Vp, self.config.d_model, lda=h16.stride(0), ldb=self.config.d_model,
               ldc=self.Vp, flags=F.GEMM_ROUND, algo_N=self.config.vocab_size)
        return out

    # ------------------------------------------------------------------ HF-style forward
    def __call__(self, input_features=None, decoder_input_ids=None, labels=None, encoder_outputs=None,
                 conv_input=None, **kw) -> Seq2SeqOutput:
        cfg = self.config
        if encoder_outputs is not None:
            enc = encoder_outputs.last_hidden_state if hasattr(encoder_outputs, "last_hidden_state") \
                else encoder_outputs[0]
            B = enc.shape[0]
            enc16 = enc.reshape(-1, cfg.d_model).to(self.device, self.act_dtype).contiguous()
            Tk = enc.shape[1]
        else:
            if conv_input is None:
                conv_input = self.conv_input(input_features)
            enc16 = self.encode(conv_input)
            B = conv_input.shape[0]
            Tk = enc16.shape[0] // B
        if decoder_input_ids is None:
            if labels is None:
                raise ValueError("need decoder_input_ids or labels")
            lab = labels.to(self.device)
            decoder_input_ids = torch.empty_like(lab)
            F.shift_tokens_right(lab.contiguous(), decoder_input_ids, cfg.pad_token_id, cfg.decoder_start_token_id)
        ids = decoder_input_ids.to(self.device)
        T = ids.shape[1]
        h = self.decode(ids, enc16, Tk)
        lp = self.lm_head(h)
        loss = None
        if labels is not None:
            lab = labels.to(self.device).reshape(-1).contiguous()
            nv = torch.zeros(1, dtype=torch.int32, device=self.device)
            F.count_valid(lab, nv)
            out3, _ = F.kl_ce(lp, lp, lab, cfg.vocab_size, nv, T=1.0, ce_w=1.0, kl_w=0.0)
            loss = out3[1]
        logits = lp.view(B, T, self.Vp)[:, :, : cfg.vocab_size]
        return Seq2SeqOutput(loss=loss, logits=logits, encoder_last_hidden_state=enc16.view(B, Tk, cfg.d_model),
                             logits_padded=lp)

    forward = __call__

    def generate(self, input_features=None, **kw):
        """Greedy (or, num_beams > 1, beam-search) decoding with a KV cache (tw/generation.py)."""
        from .generation import generate
        return generate(self, input_features, **kw)


# =============================================================================================
# backward (student).  Walks a forward tape in reverse; every weight / bias gradient is
# accumulated straight into the flat fp32 gradient buffer (model.grad) with autocast's rounding
# points: weight/bias grads of bf16 Linears are rounded to bf16 before the fp32 accumulate
# (the grad of the autocast weight cast), activation grads entering a bf16 tensor are rounded.
# =============================================================================================
def _half(x: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    out = torch.empty(x.shape, dtype=dtype, device=x.device)
    F.cast_bf16(x.contiguous(), out)
    return out


class Backward:
    def __init__(self, model: WhisperForConditionalGeneration):
        self.m = model
        self.dev = model.device
        self._ln_ws = None
        # on_ready(prefix): called once every gradient of the layer `prefix` (e.g.
        # "model.decoder.layers.1.") is final, so the DP exchange of that range can start while the
        # rest of the backward runs
        self.on_ready = None
        # (dx, g): the 16-bit copy of the stream gradient dx written by the LayerNorm backward that produced dx's
        # current value (the autocast cast the next block's GEMMs read), taken by _grad16
        self._g16 = None

    def _layer_done(self, p):
        if self.on_ready is not None and p.endswith(".self_attn"):
            self.on_ready(p[: -len("self_attn")])

    # dW[N][K] += bf16(g^T x): g [M][N] bf16, x [M][K] bf16
    def dW(self, g, x, dw, M):
        if dw is None:
            return
        N, K = dw.shape
        F.gemm(g, x, dw, N, K, M, lda=g.stride(0), ldb=x.stride(0), ldc=K, a_trans=True, b_trans=True,
               flags=F.GEMM_ROUND | F.GEMM_ACCUM)

    # dX[M][K] = op(g[M][N] W[N][K])
    # Training-sized products with the plain rounding epilogue (16-bit operands, M >= 4096, no accumulate / GELU
    # derivative) transpose W into a K-major copy first and take the forward route (persistent 256² kernel / whole-
    # round + tail split): W is read and written once more (7-33 us) and the product runs 3-23 % faster
    # (tools/bench_dx.py: whisper-small encoder QKV dX 248 -> 192 us, distil-32-2 decoder fc1 446 -> 378 us;
    # profiles/r04_m_dx_route.log).  The accumulating and GELU-derivative products keep the transposed-operand kernel:
    # on the forward route they run the persistent kernel's generic epilogue, and routing every dX measured c2 -0.8 %
    # (profiles/r04_n_dx_route_step_ab.log).  The fp32 compute path keeps the transposed-operand form.
    def dX(self, g, w, out, flags=F.GEMM_ROUND, aux=None, M=None):
        M = g.shape[0] if M is None else M
        N, K = w.shape
        if (M >= 4096 and flags == F.GEMM_ROUND and aux is None and w.dtype in F.HALF and g.dtype == w.dtype
                and out.dtype == w.dtype):
            wt = F.transpose_bf16(w, torch.empty(K, N, dtype=w.dtype, device=self.dev))
            F.gemm(g, wt, out, M, K, N, lda=g.stride(0), ldb=N, ldc=out.stride(0), flags=flags)
        else:
            F.gemm(g, w, out, M, K, N, lda=g.stride(0), ldb=K, ldc=out.stride(0), b_trans=True, aux=aux,
                   ldaux=aux.stride(0) if aux is not None else 0, flags=flags)
        return out

    def db(self, g, cols_slice, out):
        if out is None:
            return
        lo, hi = cols_slice
        F.colsum(g[:, lo:] if lo else g, g.stride(0), g.shape[0], hi - lo, out, accum=True,
                 round_bf16={"fp32": 0, "fp16": 2}.get(self.m.compute, 1))

    def ln(self, sv, name, dy, dx):
        """dx += LayerNorm backward; on the 16-bit paths the kernel also writes dx's autocast rounding (_grad16)."""
        x, mean, rstd, _ = sv[name]
        m = self.m
        D = x.shape[-1]
        need = min(1024, (x.shape[0] + 3) // 4) * 2 * D
        if self._ln_ws is None or self._ln_ws.numel() < need:
            self._ln_ws = torch.empty(need, dtype=torch.float32, device=self.dev)
        g16 = torch.empty(dx.shape, dtype=m.act_dtype, device=self.dev) if m.compute != "fp32" and _LN_G16 else None
        F.layernorm_bwd(x, m.ln_param(name + ".weight"), mean, rstd, dy, dx, m.gv(name + ".weight"),
                        m.gv(name + ".bias"), dx_accum=True, workspace=self._ln_ws, g16=g16)
        self._g16 = (dx, g16) if g16 is not None else None

    def _grad16(self, dx):
        """The stream gradient as the block's GEMMs read it (m.act_grad(dx)): the LayerNorm backward's fused copy when it
        wrote dx's current value, else a cast."""
        c, self._g16 = self._g16, None
        if c is not None and c[0] is dx:
            return c[1]
        return self.m.act_grad(dx)

    def span_grad(self, first, last, shape):
        m = self.m
        if m.gv(first) is None:
            return None
        return m.store.span(m.grad, first, last, shape)

    # ------------------------------------------------------------------
    def mlp(self, p, st, dx):
        m = self.m
        g = self._grad16(dx)
        M = g.shape[0]
        self.dW(g, st["h"], m.gv(p + ".fc2.weight"), M)
        self.db(g, (0, g.shape[1]), m.gv(p + ".fc2.bias"))
        f = st["h"].shape[1]
        dpre = torch.empty(M, f, dtype=m.act_dtype, device=self.dev)
        self.dX(g, m._w16(p + ".fc2.weight"), dpre, flags=F.GEMM_ROUND | F.GEMM_DGELU, aux=st["pre"])
        self.dW(dpre, st["y"], m.gv(p + ".fc1.weight"), M)
        self.db(dpre, (0, f), m.gv(p + ".fc1.bias"))
        dy = torch.empty(M, m.config.d_model, dtype=m.act_dtype, device=self.dev)
        self.dX(dpre, m._w16(p + ".fc1.weight"), dy)
        self.ln(st["sv"], p + ".final_layer_norm", dy, dx)

    def attn(self, p, st, dx):
        m = self.m
        d = m.config.d_model
        H = d // 64
        B, T = st["B"], st["T"]
        M = B * T
        g = self._grad16(dx)
        self.dW(g, st["o"], m.gv(p + ".out_proj.weight"), M)
        self.db(g, (0, d), m.gv(p + ".out_proj.bias"))
        do = torch.empty(M, d, dtype=m.act_dtype, device=self.dev)
        self.dX(g, m._w16(p + ".out_proj.weight"), do)
        qkv = st["qkv"]
        dqkv = torch.empty(M, 3 * d, dtype=m.act_dtype, device=self.dev)
        F.attn_bwd(qkv, 3 * d, qkv[:, d:], 3 * d, qkv[:, 2 * d:], 3 * d, st["o"], d, do, d, st["lse"], dqkv, 3 * d,
                   dqkv[:, d:], 3 * d, dqkv[:, 2 * d:], 3 * d, B, H, T, T, st["causal"], 0.125)
        self.dW(dqkv, st["y"], self.span_grad(p + ".q_proj.weight", p + ".v_proj.weight", (3 * d, d)), M)
        self.db(dqkv, (0, d), m.gv(p + ".q_proj.bias"))
        self.db(dqkv, (2 * d, 3 * d), m.gv(p + ".v_proj.bias"))
        dy = torch.empty(M, d, dtype=m.act_dtype, device=self.dev)
        wqkv = m.wspan(p + ".q_proj.weight", p + ".v_proj.weight", (3 * d, d))
        self.dX(dqkv, wqkv, dy)
        self.ln(st["sv"], p + "_layer_norm", dy, dx)

    def cross(self, p, st, dx, enc16, d_enc):
        m = self.m
        d = m.config.d_model
        H = d // 64
        B, T, Tk = st["B"], st["T"], st["Tk"]
        M = B * T
        g = self._grad16(dx)
        self.dW(g, st["o"], m.gv(p + ".out_proj.weight"), M)
        self.db(g, (0, d), m.gv(p + ".out_proj.bias"))
        do = torch.empty(M, d, dtype=m.act_dtype, device=self.dev)
        self.dX(g, m._w16(p + ".out_proj.weight"), do)
        kv = st["kv"]
        dq = torch.empty(M, d, dtype=m.act_dtype, device=self.dev)
        dkv = torch.empty(B * Tk, 2 * d, dtype=m.act_dtype, device=self.dev)
        F.attn_bwd(st["q"], d, kv, 2 * d, kv[:, d:], 2 * d, st["o"], d, do, d, st["lse"], dq, d, dkv, 2 * d,
                   dkv[:, d:], 2 * d, B, H, T, Tk, False, 0.125)
        self.dW(dq, st["y"], m.gv(p + ".q_proj.weight"), M)
        self.db(dq, (0, d), m.gv(p + ".q_proj.bias"))
        dy = torch.empty(M, d, dtype=m.act_dtype, device=self.dev)
        self.dX(dq, m._w16(p + ".q_proj.weight"), dy)
        self.ln(st["sv"], p + "_layer_norm", dy, dx)
        self.dW(dkv, enc16, self.span_grad(p + ".k_proj.weight", p + ".v_proj.weight", (2 * d, d)), B * Tk)
        self.db(dkv, (d, 2 * d), m.gv(p + ".v_proj.bias"))
        if d_enc is not None:
            wkv = m.wspan(p + ".k_proj.weight", p + ".v_proj.weight", (2 * d, d))
            self.dX(dkv, wkv, d_enc, flags=F.GEMM_ROUND | F.GEMM_ACCUM)

    # ------------------------------------------------------------------
    def decoder(self, tape, dlogits, h16, enc16, d_enc=None):
        """dlogits [M, Vp] bf16 -> accumulates every decoder / embedding gradient (and d_enc)."""
        m = self.m
        d = m.config.d_model
        M = h16.shape[0]
        E16 = m._w16("model.decoder.embed_tokens.weight")
        gE = m.gv("model.decoder.embed_tokens.weight")
        # LM head (tied): dh = e(dlogits E), dE += e(dlogits^T h) (e = the autocast dtype).  On the 16-bit paths E goes
        # K-major first (one 133 MB transpose): the K = 51 904 product then runs on the persistent kernel
        dh = torch.empty(M, d, dtype=m.act_dtype, device=self.dev)
        if E16.dtype in F.HALF and M >= 4096:
            ET = F.transpose_bf16(E16, torch.empty(d, m.Vp, dtype=E16.dtype, device=self.dev))
            F.gemm(dlogits, ET, dh, M, d, m.Vp, lda=m.Vp, ldb=m.Vp, ldc=d, flags=F.GEMM_ROUND)
            del ET
        else:
            F.gemm(dlogits, E16, dh, M, d, m.Vp, lda=m.Vp, ldb=d, ldc=d, b_trans=True, flags=F.GEMM_ROUND)
        if gE is not None:
            F.gemm(dlogits, h16, gE, m.Vp, d, M, lda=m.Vp, ldb=d, ldc=d, a_trans=True, b_trans=True,
                   flags=F.GEMM_ROUND | F.GEMM_ACCUM)
        dx = torch.zeros(M, d, dtype=torch.float32, device=self.dev)
        for kind, p, st in reversed(tape):
            if kind == "ln_final":
                self.ln(st["sv"], p, dh, dx)
            elif kind == "mlp":
                self.mlp(p, st, dx)
            elif kind == "cross":
                self.cross(p, st, dx, enc16, d_enc)
            elif kind == "attn":
                self.attn(p, st, dx)
                self._layer_done(p)
            elif kind == "embed":
                if gE is not None:
                    # HF's decoder embed_tokens has padding_idx = pad_token_id: pad positions add nothing
                    F.embed_bwd(st["ids"], dx, gE, padding_idx=m.config.pad_token_id)
                gP = m.gv("model.decoder.embed_positions.weight")
                if gP is not None:   # sum over the batch of position rows
                    F.colsum(dx, st["T"] * d, st["B"], st["T"] * d, gP.view(-1), accum=True, round_bf16=False)
        return dx

    def encoder(self, tape, d_enc):
        """d_enc [B*1500, d] fp32 (grad of encoder_last_hidden_state) -> encoder grads."""
        m = self.m
        d = m.config.d_model
        dx = torch.zeros_like(d_enc)
        for kind, p, st in reversed(tape):
            if kind == "ln_final":
                self.ln(st["sv"], p, d_enc, dx)
            elif kind == "mlp":
                self.mlp(p, st, dx)
            elif kind == "attn":
                self.attn(p, st, dx)
                self._layer_done(p)
            elif kind == "conv":
                self.conv(st, dx)

    def conv(self, st, dx0):
        m = self.m
        cfg, d = m.config, m.config.d_model
        B, T = st["B"], st["T"]
        T2, nm = 2 * T, cfg.num_mel_bins
        g1w, g2w = m.gv("model.encoder.conv1.weight"), m.gv("model.encoder.conv2.weight")
        if g1w is None and g2w is None:
            return
        dpre2 = torch.empty(B * T, d, dtype=m.act_dtype, device=self.dev)
        F.gelu_bwd(dx0, st["pre2"].view(B * T, d), dpre2)
        A2 = torch.empty(B * T, 3 * d, dtype=m.act_dtype, device=self.dev)
        F.im2col3(st["H1"], T2 + 2, A2, B, T, 2, d)
        self.dW(dpre2, A2, g2w, B * T)
        self.db(dpre2, (0, d), m.gv("model.encoder.conv2.bias"))
        dA2 = torch.empty(B * T, 3 * d, dtype=torch.float32, device=self.dev)
        self.dX(dpre2, m._w16("model.encoder.conv2.weight"), dA2, flags=0)
        dH1 = torch.empty(B * T2, d, dtype=torch.float32, device=self.dev)
        F.col2im_s2(dA2, dH1, B, T2, T, d)
        dpre1 = torch.empty(B * T2, d, dtype=m.act_dtype, device=self.dev)
        F.gelu_bwd(dH1, st["pre1"].view(B * T2, d), dpre1)
        A1 = torch.empty(B * T2, 3 * nm, dtype=m.act_dtype, device=self.dev)
        F.im2col3(st["conv_in"], T2 + 2, A1, B, T2, 1, nm)
        self.dW(dpre1, A1, g1w, B * T2)
        self.db(dpre1, (0, d), m.gv("model.encoder.conv1.bias"))


def random_init_(model: WhisperForConditionalGeneration, seed: int = 0, std: float = 0.02):
    """Random weights of the right architecture on the device (benchmarks: no checkpoints offline).
    LayerNorm = (1, 0), encoder positions = sinusoids (what checkpoints carry), pad rows 0."""
    cfg = model.config
    g = torch.Generator(device=model.device).manual_seed(seed)
    st = model.store
    buf = st.p32 if st.p32 is not None else st.p16
    for n in st.order:
        v = st._view(buf, n)
        if is_pseudo(n) or n.endswith("bias"):
            v.zero_()
        elif "layer_norm" in n:
            v.fill_(1.0)
        elif n.endswith("encoder.embed_positions.weight"):
            L, d = v.shape
            inc = math.log(10000.0) / (d // 2 - 1)
            inv = torch.exp(-inc * torch.arange(d // 2, device=model.device, dtype=torch.float32))
            tt = torch.arange(L, device=model.device, dtype=torch.float32)[:, None] * inv[None, :]
            v.copy_(torch.cat([tt.sin(), tt.cos()], 1))
        else:
            v.copy_(torch.randn(v.shape, generator=g, device=model.device) * std)
            if n.endswith("embed_tokens.weight"):
                v[cfg.vocab_size:].zero_()
    if st.p32 is not None:
        F.cast_bf16(st.p32, st.p16)
    model._refresh_ln32()
    return model
