"""Greedy generation with a KV cache.

Reference calls: `generate_step` (training/run_distillation.py:1580-1584), pseudo-labelling
`generate(num_beams=1, language, task)` (training/run_pseudo_labelling.py:917-922); semantics of
HF WhisperForConditionalGeneration.generate greedy path (HF generation_whisper.py): prompt
[<|startoftranscript|>, <|lang|>, <|task|>, <|notimestamps|>], SuppressTokens every step,
SuppressTokensAtBegin at the first generated step (HF logits_process.py), argmax, finished rows
padded with pad (= eos), stop when every row emitted eos or max_length is reached; the return
value is the generated ids only (transformers >= 5 behaviour, the version in this image).

Device layout (one DecodeSession per batch of clips):
  * self-attention cache per decoder layer: bf16 [B][T_max][2d] (k | v); the fused QKV projection
    of a step goes to a [B][3d] staging buffer and tw_kv_append copies k, v to row t; keys /
    values 0..t are read in place by tw_decode_attn;
  * cross-attention K/V per decoder layer: bf16 [B*1500][2d], projected once from the encoder
    output (k has no bias: the zero-bias segment of the fused KV bias);
  * logits bf16 [B][Vp]; tw_greedy_select applies the suppress masks, takes the argmax, writes
    the token into the id matrix and the next step's input vector, and tracks finished rows.
Everything runs on the HIP library.  The step index lives in device memory (t_dev: embedding
position, cache row, self-attention length, output column, begin-suppress test), so one step —
~14 launches per decoder layer + head + select + advance — is captured once into a HIP graph and
replayed per token; the host reads the finished flags every 8 steps to stop early.
"""
from __future__ import annotations

import torch

from . import ops as F


class DecodeSession:
    """Device state of one greedy decode over a batch; every step is position-independent (the step
    index lives in `t_dev`), so the whole step is captured once into a HIP graph and replayed."""

    def __init__(self, model, enc16: torch.Tensor, B: int, Tk: int, T_max: int):
        cfg = model.config
        self.m, self.B, self.Tk, self.T_max = model, B, Tk, T_max
        self.d = cfg.d_model
        self.H = self.d // 64
        dev = model.device
        d = self.d
        self.self_kv = [torch.empty(B, T_max, 2 * d, dtype=torch.bfloat16, device=dev)
                        for _ in range(cfg.decoder_layers)]
        self.cross_kv = []
        for i in range(cfg.decoder_layers):
            p = f"model.decoder.layers.{i}.encoder_attn"
            kv = torch.empty(B * Tk, 2 * d, dtype=torch.bfloat16, device=dev)
            wkv = model.store.span(model.store.p16, p + ".k_proj.weight", p + ".v_proj.weight", (2 * d, d))
            bkv = model.store.span(model.store.p16, p + ".k_proj.zero_bias", p + ".v_proj.bias", (2 * d,))
            model._lin(enc16, wkv, bkv, kv)
            self.cross_kv.append(kv)
        self.t_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.cur = torch.zeros(B, dtype=torch.int64, device=dev)       # this step's input ids
        self.x = torch.empty(B, d, dtype=model.stream_dtype, device=dev)
        self.y = torch.empty(B, d, dtype=torch.bfloat16, device=dev)
        self.qkv = torch.empty(B, 3 * d, dtype=torch.bfloat16, device=dev)
        self.o = torch.empty(B, d, dtype=torch.bfloat16, device=dev)
        self.q = torch.empty(B, d, dtype=torch.bfloat16, device=dev)
        self.h = torch.empty(B, cfg.decoder_ffn_dim, dtype=torch.bfloat16, device=dev)
        self.logits = torch.empty(B, model.Vp, dtype=torch.bfloat16, device=dev)
        self.graph = None

    def _ln(self, x, name):
        m = self.m
        F.layernorm_fwd(x, m.ln_param(name + ".weight"), m.ln_param(name + ".bias"), self.y)
        return self.y

    def step(self, select=None):
        """One decoder step at position *t_dev for input ids `cur`; then t_dev += 1.
        select = (sup, beg, eos, done, ids, P) runs greedy selection into ids[:, t+1] and cur."""
        m, B, d, H, T_max = self.m, self.B, self.d, self.H, self.T_max
        if m.store.p32 is not None:
            E, Pe = m.store.v32("model.decoder.embed_tokens.weight"), m.store.v32("model.decoder.embed_positions.weight")
        else:
            E, Pe = m.store.v16("model.decoder.embed_tokens.weight"), m.store.v16("model.decoder.embed_positions.weight")
        x, o, t_dev = self.x, self.o, self.t_dev
        F.embed_step(self.cur, E, Pe, x, t_dev, T_max)
        sb = T_max * 2 * d
        for i in range(m.config.decoder_layers):
            p = f"model.decoder.layers.{i}"
            # self attention: fused QKV -> staging; k, v appended at row t of the cache
            y = self._ln(x, p + ".self_attn_layer_norm")
            wqkv = m.store.span(m.store.p16, p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight",
                                (3 * d, d))
            bqkv = m.store.span(m.store.p16, p + ".self_attn.q_proj.bias", p + ".self_attn.v_proj.bias", (3 * d,))
            m._lin(y, wqkv, bqkv, self.qkv)
            cache = self.self_kv[i]
            F.kv_append(self.qkv[:, d:], 3 * d, cache, 2 * d, sb, B, 2 * d, t_dev, T_max)
            F.decode_attn(self.qkv, 3 * d, cache, 2 * d, sb, cache.view(-1)[d:], 2 * d, sb, o, d, B, H, 1, 0.125,
                          tk_dev=t_dev, tk_max=T_max)
            m._lin(o, m._w16(p + ".self_attn.out_proj.weight"), m._w16(p + ".self_attn.out_proj.bias"), x, res=x)
            # cross attention over the encoder frames
            y = self._ln(x, p + ".encoder_attn_layer_norm")
            m._lin(y, m._w16(p + ".encoder_attn.q_proj.weight"), m._w16(p + ".encoder_attn.q_proj.bias"), self.q)
            kv = self.cross_kv[i]
            F.decode_attn(self.q, d, kv, 2 * d, self.Tk * 2 * d, kv[:, d:], 2 * d, self.Tk * 2 * d, o, d, B, H,
                          self.Tk, 0.125)
            m._lin(o, m._w16(p + ".encoder_attn.out_proj.weight"), m._w16(p + ".encoder_attn.out_proj.bias"), x,
                   res=x)
            # MLP
            y = self._ln(x, p + ".final_layer_norm")
            m._lin(y, m._w16(p + ".fc1.weight"), m._w16(p + ".fc1.bias"), self.h, flags=F.GEMM_ROUND | F.GEMM_GELU)
            m._lin(self.h, m._w16(p + ".fc2.weight"), m._w16(p + ".fc2.bias"), x, res=x)
        hN = self._ln(x, "model.decoder.layer_norm")
        m.lm_head(hN, out=self.logits)
        if select is not None:
            sup, beg, eos, done, ids, P = select
            F.greedy_select(self.logits, m.Vp, B, m.config.vocab_size, sup, beg, False, eos, done, ids, 1, self.cur,
                            t_dev=t_dev, begin_col=P)
        F.step_advance(t_dev)

    def capture(self, select):
        """Record one selecting step into a HIP graph (nothing executes during capture)."""
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.step(select)
        self.graph = g


def _lang_id(gc, language):
    if language is None:
        return None
    if isinstance(language, int):
        return language
    l2i = dict(gc.lang_to_id or {})
    for key in (language, f"<|{language}|>"):
        if key in l2i:
            return l2i[key]
    builtin = {"en": 50259, "zh": 50260}
    lang = language.strip("<|>")
    if lang in builtin:
        return builtin[lang]
    raise ValueError(f"unknown language {language!r} (generation_config.lang_to_id has {sorted(l2i)[:5]}...)")


def build_prompt(gc, language=None, task=None, return_timestamps=False):
    """HF Whisper prompt: [SOT, <|lang|>, <|task|>, (<|notimestamps|>)] (generation_whisper.py)."""
    ids = [gc.decoder_start_token_id]
    lid = _lang_id(gc, language)
    if lid is not None:
        ids.append(lid)
    if task is not None or lid is not None:
        ids.append(dict(gc.task_to_id or {}).get(task or "transcribe", 50359))
    if not return_timestamps:
        ids.append(gc.no_timestamps_token_id)
    return ids


@torch.no_grad()
def generate(model, input_features=None, max_length=None, num_beams=1, return_timestamps=False, language=None,
             task=None, decoder_input_ids=None, max_new_tokens=None, encoder_outputs=None, attention_mask=None,
             use_graph=None, **kw):
    from .config import GenerationConfig
    if num_beams not in (None, 1):
        raise NotImplementedError("tw generate: greedy only (num_beams=1, as every reference call site)")
    if kw.get("do_sample"):
        raise NotImplementedError("tw generate: sampling is not on the hot path")
    if return_timestamps:
        raise NotImplementedError("tw generate: timestamp decoding is SURVEY.md §8f item 3 (long-form), not built")
    gc = model.generation_config if model.generation_config is not None else GenerationConfig()
    if not isinstance(gc, GenerationConfig):
        gc = GenerationConfig(gc)
    cfg = model.config
    if encoder_outputs is not None:
        enc = encoder_outputs.last_hidden_state if hasattr(encoder_outputs, "last_hidden_state") else encoder_outputs[0]
        B, Tk = enc.shape[0], enc.shape[1]
        enc16 = enc.reshape(-1, cfg.d_model).to(model.device, torch.bfloat16).contiguous()
    else:
        conv_in = model.conv_input(input_features)
        enc16 = model.encode(conv_in)
        B = conv_in.shape[0]
        Tk = enc16.shape[0] // B
    if decoder_input_ids is not None:
        prompt = torch.as_tensor(decoder_input_ids, dtype=torch.int64)
        if prompt.dim() == 1:
            prompt = prompt[None].repeat(B, 1)
    else:
        prompt = torch.tensor(build_prompt(gc, language, task, return_timestamps), dtype=torch.int64)[None].repeat(B, 1)
    P = prompt.shape[1]
    if max_new_tokens is not None:
        max_length = P + int(max_new_tokens)
    if max_length is None:
        max_length = gc.max_length or cfg.max_target_positions
    max_length = min(int(max_length), cfg.max_target_positions)
    if P >= max_length:
        return torch.empty(B, 0, dtype=torch.int64, device=model.device)
    dev = model.device
    eos = int(gc.eos_token_id if gc.eos_token_id is not None else cfg.eos_token_id)
    V = cfg.vocab_size
    ids = torch.full((B, max_length), eos, dtype=torch.int64, device=dev)
    ids[:, :P] = prompt.to(dev)
    done = torch.zeros(B, dtype=torch.uint8, device=dev)
    sup = F.token_bitmask(gc.suppress_tokens or [], V, dev)
    beg = F.token_bitmask(gc.begin_suppress_tokens or [], V, dev)
    sess = DecodeSession(model, enc16, B, Tk, max_length)
    for t in range(P - 1):                                   # prefill the cache with the prompt
        sess.cur.copy_(ids[:, t])
        sess.step()
    sess.cur.copy_(ids[:, P - 1])
    select = (sup, beg, eos, done, ids, P)
    graph = use_graph if use_graph is not None else True
    if graph:
        sess.capture(select)
    t = P - 1
    while t + 1 < max_length:
        if graph:
            sess.graph.replay()
        else:
            sess.step(select)
        t += 1
        if (t - P) % 8 == 7 and bool(done.all()):
            break
    gen = ids[:, P:t + 1]
    # trim trailing columns in which every row had already finished (HF stops at the step
    # where the last row emits eos)
    is_eos = (gen == eos).cpu()
    first = torch.where(is_eos.any(1), is_eos.int().argmax(1), torch.full((B,), gen.shape[1]))
    L = int(min(gen.shape[1], int(first.max()) + 1)) if B else 0
    return gen[:, :L]
