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

import os
import time

import torch

from . import ops as F

_XKV_HEAD_MAJOR = os.environ.get("TW_XKV_HEAD_MAJOR", "1") != "0"


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
        act = model.act_dtype            # bf16 (autocast) or fp32 (fp32 path): caches, operands, logits
        self.self_kv = [torch.empty(B, T_max, 2 * d, dtype=act, device=dev)
                        for _ in range(cfg.decoder_layers)]
        # cross-attention K/V head-major (K [B][H][Tk][64] then V): each (clip, head) of the per-step
        # cross-attention reads two contiguous runs instead of 128-B rows 2d apart (tw_kv_head_major; the
        # projection goes through one scratch [B*Tk][2d] block).  TW_XKV_HEAD_MAJOR=0: the projection's own
        # row-interleaved layout (A/B runs).
        self.hm = _XKV_HEAD_MAJOR
        if self.hm:
            self.cross_kv = [torch.empty(2 * B * self.H * Tk * 64, dtype=act, device=dev)
                             for _ in range(cfg.decoder_layers)]
        else:
            self.cross_kv = [torch.empty(B * Tk, 2 * d, dtype=act, device=dev)
                             for _ in range(cfg.decoder_layers)]
        self.graph = None
        self.xkv_shared = False
        self.set_encoder(enc16)
        self.t_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.cur = torch.zeros(B, dtype=torch.int64, device=dev)       # this step's input ids
        self.x = torch.empty(B, d, dtype=model.stream_dtype, device=dev)
        self.y = torch.empty(B, d, dtype=act, device=dev)
        self.qkv = torch.empty(B, 3 * d, dtype=act, device=dev)
        self.o = torch.empty(B, d, dtype=act, device=dev)
        self.q = torch.empty(B, d, dtype=act, device=dev)
        self.h = torch.empty(B, cfg.decoder_ffn_dim, dtype=act, device=dev)
        self.logits = torch.empty(B, model.Vp, dtype=act, device=dev)
        # batch <= 8 on the bf16 / fp16 paths: every Linear is one GEMV launch, with the LayerNorm in front of it
        # fused when the residual stream is 16-bit (bit-identical A); larger batches use the skinny GEMM with a
        # separate LayerNorm
        self.gemv = B <= 8 and model.compute in ("bf16", "fp16") and d % 256 == 0
        self.gemv_ln = self.gemv and model.stream_dtype == act

    def set_encoder(self, enc16):
        """(Re)project the cross-attention K/V of every decoder layer in place (graph-safe).  enc16 holds B*Tk
        rows, or Tk rows shared by every row of the batch (the speculative fallback batch of one window: the
        K/V are projected once and copied, so each row sees exactly the K/V of a batch-1 decode)."""
        m, d = self.m, self.d
        shared = enc16.shape[0] == self.Tk and self.B > 1
        nb = 1 if shared else self.B
        # head-major and shared: ONE clip's K/V blocks ([H][Tk][64] K then V, at the front of each layer's buffer),
        # read by every row with batch stride 0 (tw_decode_attn_hs) instead of B copies: the fallback batch's
        # cross-attention reads 1/B of the bytes and each row still sees exactly its batch-1 K/V.  The captured step
        # bakes the call's strides in, so a change of mode drops the graph (recaptured on the next run)
        xs = self.hm and shared
        if self.graph is not None and xs != self.xkv_shared:
            self.graph = None
        self.xkv_shared = xs
        # head-major: the projection goes through one [B*Tk][2d] scratch block that lives only for this call
        # (3.9 GB at the 512-clip large-v2 batch; the caching allocator reuses it for the next window)
        proj = torch.empty(nb * self.Tk, 2 * d, dtype=m.act_dtype, device=m.device) if self.hm or shared else None
        for i, kv in enumerate(self.cross_kv):
            p = f"model.decoder.layers.{i}.encoder_attn"
            wkv = m.wspan(p + ".k_proj.weight", p + ".v_proj.weight", (2 * d, d))
            bkv = m.wspan(p + ".k_proj.zero_bias", p + ".v_proj.bias", (2 * d,))
            if self.hm and shared:               # K [H][Tk][64] then V of the one clip, shared by every row
                m._lin(enc16, wkv, bkv, proj)
                F.kv_head_major(proj, 2 * d, kv, 1, self.Tk, self.H)
            elif self.hm:
                m._lin(enc16, wkv, bkv, proj)
                F.kv_head_major(proj, 2 * d, kv, nb, self.Tk, self.H)
            elif shared:
                m._lin(enc16, wkv, bkv, proj)
                kv.view(self.B, self.Tk, 2 * d).copy_(proj.view(1, self.Tk, 2 * d).expand(self.B, -1, -1))
            else:
                m._lin(enc16, wkv, bkv, kv)
        del proj

    def _ln(self, x, name):
        m = self.m
        F.layernorm_fwd(x, m.ln_param(name + ".weight"), m.ln_param(name + ".bias"), self.y)
        return self.y

    def _ln_lin(self, x, ln, w, b, out, flags=F.GEMM_ROUND, kv=None):
        """out = Linear(LayerNorm(x)): one GEMV launch (batch <= 4, bf16 stream) or LN + GEMM.  kv: the
        GEMV also appends columns >= kv[3] to the self-attention cache row (only on the GEMV path)."""
        m = self.m
        if self.gemv_ln:
            F.gemv(x, w, out, ln_w=m.ln_param(ln + ".weight"), ln_b=m.ln_param(ln + ".bias"), bias=b, flags=flags,
                   kv=kv)
        else:
            y = self._ln(x, ln)
            if self.gemv:
                F.gemv(y, w, out, bias=b, flags=flags)
            else:
                m._lin(y, w, b, out, flags=flags)
        return out

    def _lin(self, a, w, b, out, res=None, flags=F.GEMM_ROUND):
        if self.gemv:
            F.gemv(a, w, out, bias=b, res=res, flags=flags)
        else:
            self.m._lin(a, w, b, out, res=res, flags=flags)
        return out

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
            wqkv = m.wspan(p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight", (3 * d, d))
            bqkv = m.wspan(p + ".self_attn.q_proj.bias", p + ".self_attn.v_proj.bias", (3 * d,))
            cache = self.self_kv[i]
            if self.gemv_ln:        # k, v of this step written to cache row t by the QKV GEMV itself
                self._ln_lin(x, p + ".self_attn_layer_norm", wqkv, bqkv, self.qkv, kv=(cache, sb, 2 * d, d, t_dev,
                                                                                     T_max))
            else:
                self._ln_lin(x, p + ".self_attn_layer_norm", wqkv, bqkv, self.qkv)
                F.kv_append(self.qkv[:, d:], 3 * d, cache, 2 * d, sb, B, 2 * d, t_dev, T_max)
            F.decode_attn(self.qkv, 3 * d, cache, 2 * d, sb, cache.view(-1)[d:], 2 * d, sb, o, d, B, H, 1, 0.125,
                          tk_dev=t_dev, tk_max=T_max)
            self._lin(o, m._w16(p + ".self_attn.out_proj.weight"), m._w16(p + ".self_attn.out_proj.bias"), x, res=x)
            # cross attention over the encoder frames
            self._ln_lin(x, p + ".encoder_attn_layer_norm", m._w16(p + ".encoder_attn.q_proj.weight"),
                         m._w16(p + ".encoder_attn.q_proj.bias"), self.q)
            kv = self.cross_kv[i]
            if self.xkv_shared:     # every row over the one clip's [H][Tk][64] blocks (batch stride 0)
                n1 = H * self.Tk * 64
                F.decode_attn(self.q, d, kv, 64, 0, kv[n1:], 64, 0, o, d, B, H, self.Tk, 0.125, hsk=self.Tk * 64,
                              hsv=self.Tk * 64)
            elif self.hm:         # B*H one-head clips over contiguous [Tk][64] runs
                hv = B * H * self.Tk * 64
                F.decode_attn(self.q, 64, kv, 64, self.Tk * 64, kv[hv:], 64, self.Tk * 64, o, 64, B * H, 1,
                              self.Tk, 0.125)
            else:
                F.decode_attn(self.q, d, kv, 2 * d, self.Tk * 2 * d, kv[:, d:], 2 * d, self.Tk * 2 * d, o, d, B, H,
                              self.Tk, 0.125)
            self._lin(o, m._w16(p + ".encoder_attn.out_proj.weight"), m._w16(p + ".encoder_attn.out_proj.bias"), x,
                      res=x)
            # MLP
            self._ln_lin(x, p + ".final_layer_norm", m._w16(p + ".fc1.weight"), m._w16(p + ".fc1.bias"), self.h,
                         flags=F.GEMM_ROUND | F.GEMM_GELU)
            self._lin(self.h, m._w16(p + ".fc2.weight"), m._w16(p + ".fc2.bias"), x, res=x)
        if self.gemv_ln:
            self._ln_lin(x, "model.decoder.layer_norm", m._w16("model.decoder.embed_tokens.weight"), None,
                         self.logits)
        else:
            m.lm_head(self._ln(x, "model.decoder.layer_norm"), out=self.logits)
        if select is not None:
            select(self)
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


class _Select:
    """Per-step token selection into ids[:, t+1] (t read on the device): HF SuppressTokens,
    SuppressTokensAtBegin and, with timestamps, WhisperTimeStampLogitsProcessor + argmax."""

    def __init__(self, gc, B, V, T_max, P, dev, timestamps, track=False):
        self.V, self.P, self.ts, self.track = V, P, timestamps, track
        self.eos = int(gc.eos_token_id)
        self.sup = F.token_bitmask(gc.suppress_tokens or [], V, dev)
        self.beg = F.token_bitmask(gc.begin_suppress_tokens or [], V, dev)
        self.ids = torch.full((B, T_max), self.eos, dtype=torch.int64, device=dev)
        self.done = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.last_ts = torch.full((B,), -1, dtype=torch.int32, device=dev)
        self.no_ts = int(gc.no_timestamps_token_id)
        mi = gc.max_initial_timestamp_index if "max_initial_timestamp_index" in gc else None
        self.max_initial = -1 if mi is None else int(mi)
        # temperature fallback: one sampling control word (1/T, seed) per row, read on the device, so a captured
        # graph serves every temperature and the rows of a batch can be different fallback attempts; running
        # log-prob of the chosen tokens
        self.B = B
        self.ctl = torch.zeros(3 * B, dtype=torch.int32, device=dev) if track else None
        self.sum_logp = torch.zeros(B, dtype=torch.float32, device=dev) if track else None

    def reset(self, prompt, temperature=0.0, seed=0):
        """temperature / seed: one value for every row, or one per row."""
        self.ids.fill_(self.eos)
        self.ids[:, :self.P] = prompt
        self.done.zero_()
        self.last_ts.fill_(-1)
        temps = list(temperature) if isinstance(temperature, (list, tuple)) else [temperature] * self.B
        seeds = list(seed) if isinstance(seed, (list, tuple)) else [seed] * self.B
        if self.track:
            self.sum_logp.zero_()
            F.sample_ctl(temps, seeds, self.ctl)
        elif any(temps):
            raise ValueError("sampling needs a tracking selector (track=True)")

    def __call__(self, sess):
        B = sess.B
        if self.track:
            if self.ts:
                F.select_sample_ts(sess.logits, sess.m.Vp, B, self.V, self.sup, self.beg, self.eos, self.done, self.ids,
                                   1, sess.cur, self.last_ts, self.P, self.ctl, self.sum_logp, ts_begin=self.no_ts + 1,
                                   no_ts=self.no_ts, max_initial=self.max_initial, t_dev=sess.t_dev)
            else:
                F.select_sample(sess.logits, sess.m.Vp, B, self.V, self.sup, self.beg, False, self.eos, self.done,
                                self.ids, 1, sess.cur, self.ctl, self.sum_logp, t_dev=sess.t_dev, begin_col=self.P)
        elif self.ts:
            F.greedy_select_ts(sess.logits, sess.m.Vp, B, self.V, self.sup, self.beg, self.eos, self.done, self.ids, 1,
                               sess.cur, self.last_ts, self.P, ts_begin=self.no_ts + 1, no_ts=self.no_ts,
                               max_initial=self.max_initial, t_dev=sess.t_dev)
        else:
            F.greedy_select(sess.logits, sess.m.Vp, B, self.V, self.sup, self.beg, False, self.eos, self.done, self.ids,
                            1, sess.cur, t_dev=sess.t_dev, begin_col=self.P)


class _Decoder:
    """One greedy decode of B windows with a fixed prompt; reusable across windows (long-form):
    the captured step graph stays valid because every buffer it touches is reused in place."""

    def __init__(self, model, gc, B, Tk, P, max_length, timestamps, use_graph, track=False):
        self.m, self.P, self.T_max, self.use_graph = model, P, max_length, use_graph
        self.sess = None
        self.sel = _Select(gc, B, model.config.vocab_size, max_length, P, model.device, timestamps, track)
        self.B, self.Tk = B, Tk
        self.ns_logp = torch.zeros(B, dtype=torch.float32, device=model.device) if track else None

    def run(self, enc16, prompt, temperature=0.0, seed=0, no_speech=None):
        """prompt: int64 [B, P] (device) -> generated ids [B, L] (device), HF trimming.
        no_speech = (sot_position, token): log-softmax of the raw logits at the <|startoftranscript|>
        position for that token goes to self.ns_logp (WhisperNoSpeechDetection)."""
        sel, P = self.sel, self.P
        if self.sess is None:
            self.sess = DecodeSession(self.m, enc16, self.B, self.Tk, self.T_max)
        else:
            self.sess.set_encoder(enc16)
        sess = self.sess
        sel.reset(prompt, temperature, seed)
        sess.t_dev.zero_()
        V = self.m.config.vocab_size
        for t in range(P - 1):                                   # prefill the cache with the prompt
            sess.cur.copy_(sel.ids[:, t])
            sess.step()
            if no_speech is not None and t == no_speech[0]:
                F.token_logprob(sess.logits, self.m.Vp, self.B, V, no_speech[1], self.ns_logp)
        sess.cur.copy_(sel.ids[:, P - 1])
        if self.use_graph and sess.graph is None:
            sess.capture(sel)
        t = P - 1
        while t + 1 < self.T_max:
            if self.use_graph:
                sess.graph.replay()
            else:
                sess.step(sel)
            if no_speech is not None and t == P - 1 and no_speech[0] == P - 1:
                F.token_logprob(sess.logits, self.m.Vp, self.B, V, no_speech[1], self.ns_logp)
            t += 1
            if (t - P) % 8 == 7 and bool(sel.done.all()):
                break
        gen = sel.ids[:, P:t + 1]
        # trim trailing columns in which every row had already finished (HF stops at the step
        # where the last row emits eos)
        is_eos = (gen == sel.eos).cpu()
        B = gen.shape[0]
        first = torch.where(is_eos.any(1), is_eos.int().argmax(1), torch.full((B,), gen.shape[1]))
        L = int(min(gen.shape[1], int(first.max()) + 1)) if B else 0
        return gen[:, :L]


class _BeamDecoder:
    """Beam search over B clips x k beams with the same prompt (with `timestamps`, one window of the seek loop): HF
    GenerationMixin._beam_search (transformers 5.15 generation/utils.py:3208-3560), the search behind
    `training/run_eval.py:144-147` (--num_beams) and `run_distillation.py:1476-1484` (generation_num_beams).
    The B*k rows decode as one batch on the engine's step (DecodeSession, every clip's encoder rows repeated k
    times); per step, on the device: fp32 log-softmax of the logits, the suppress processors on the log-probs,
    plus the running scores, the top 2k of k*V candidates, the k best unfinished continue (the self-attention
    caches gathered by their source beams), finished candidates among the top k enter the per-clip set of k
    hypotheses with score sum(log p) / generated_length ** length_penalty; the search stops when no running beam
    can beat the worst kept hypothesis (early_stopping False: the heuristic at the current length) or every
    candidate hits max_length."""

    def __init__(self, model, gc, B, nb, Tk, P, max_length, timestamps=None):
        self.m, self.gc, self.B, self.nb, self.Tk, self.P, self.T_max = model, gc, B, nb, Tk, P, max_length
        # timestamps: (ts_begin, no_ts, max_initial) -> HF WhisperTimeStampLogitsProcessor on the log-probs after the
        # suppress processors (generation_whisper.py _retrieve_logit_processors order), begin_index = P; with it the
        # decoder also tracks, per hypothesis, the sum over its steps of log_softmax(processed row)[token] -- what HF's
        # _retrieve_avg_logprobs sums over the chosen beam's scores (beam_indices) for the fallback gate
        self.ts = timestamps
        self.sum_logp = None      # [B] after run(): that sum for each clip's best hypothesis
        self.ns_prob = None       # [B] after run(no_speech=...): no-speech probability (_ns)
        dev = model.device
        self.V = model.config.vocab_size
        self.eos = int(gc.eos_token_id)
        pad = getattr(gc, "pad_token_id", None)
        self.fill = int(pad) if pad is not None else self.eos
        self.sup = torch.tensor(sorted(set(gc.suppress_tokens or [])), dtype=torch.int64, device=dev)
        self.beg = torch.tensor(sorted(set(gc.begin_suppress_tokens or [])), dtype=torch.int64, device=dev)
        self.length_penalty = float(getattr(gc, "length_penalty", 1.0) if getattr(gc, "length_penalty", None)
                                    is not None else 1.0)
        es = getattr(gc, "early_stopping", False)
        self.early_stopping = False if es is None else es

    def _ns(self, sess, token):
        """WhisperNoSpeechDetection under beam search (is_scores_logprobs): exp of the fp32 log-softmax of the raw
        logits at <|startoftranscript|>, the first beam row of each clip (every beam row holds the prompt there)."""
        lg = sess.logits.view(self.B, self.nb, -1)[:, 0, :self.V].float()
        return torch.log_softmax(lg, dim=-1)[:, token].exp()

    @staticmethod
    def _gather(t, idx):
        """HF _gather_beams: t [B, K, ...] rows picked per clip by idx [B, k]."""
        while idx.dim() < t.dim():
            idx = idx.unsqueeze(-1)
        return torch.gather(t, 1, idx.expand(*idx.shape[:2], *t.shape[2:]))

    def _ts_rules(self, logp, run_seq, run_last_ts, cur):
        """HF WhisperTimeStampLogitsProcessor (transformers generation/logits_process.py) on the B*k processed
        log-prob rows, vectorised: <|notimestamps|> masked; timestamps in pairs (after a pair no timestamp, after a single
        one no text); timestamps never decrease (nor repeat <|0.00|>); the first step a timestamp <= max_initial; then
        text masked where the timestamps' summed probability beats every text token."""
        tb, no_ts, max_initial = self.ts
        eos = self.eos
        BN, V = logp.shape
        logp[:, no_ts] = -float("inf")
        ngen = cur - self.P
        cols = torch.arange(V, device=logp.device)
        if ngen >= 1:
            last = run_seq[:, :, cur - 1].reshape(-1)
            last_is = last >= tb
            pen_is = (run_seq[:, :, cur - 2].reshape(-1) >= tb) if ngen >= 2 else torch.ones_like(last_is)
            kill_ts = last_is & pen_is
            kill_text = last_is & ~pen_is
            logp.masked_fill_(kill_ts[:, None] & (cols >= tb)[None, :], -float("inf"))
            logp.masked_fill_(kill_text[:, None] & (cols < eos)[None, :], -float("inf"))
            lts = run_last_ts.reshape(-1)
            lim = torch.where(kill_text, lts, lts + 1)
            logp.masked_fill_((lts >= 0)[:, None] & (cols >= tb)[None, :] & (cols[None, :] < lim[:, None]),
                              -float("inf"))
        else:
            logp[:, :tb] = -float("inf")
            if max_initial is not None:
                logp[:, tb + max_initial + 1:] = -float("inf")
        lp2 = torch.log_softmax(logp.float(), dim=-1)
        ts_mass = torch.logsumexp(lp2[:, tb:], dim=-1)
        text_max = lp2[:, :tb].max(dim=-1).values
        logp.masked_fill_((ts_mass > text_max)[:, None] & (cols < tb)[None, :], -float("inf"))
        return logp

    def run(self, enc16, prompt, no_speech=None):
        """enc16: [B*Tk, d] encoder rows; prompt: int64 [P] (device or host) -> generated ids [B, L] (device).
        no_speech = (sot_position, token): softmax of the raw logits at that prompt position for that token goes to
        self.ns_prob (WhisperNoSpeechDetection)."""
        m, B, nb, P, T_max, V = self.m, self.B, self.nb, self.P, self.T_max, self.V
        dev = m.device
        d = m.config.d_model
        BN = B * nb
        prompt = torch.as_tensor(prompt, dtype=torch.int64, device=dev)
        enc_rep = enc16.view(B, self.Tk, d).repeat_interleave(nb, 0).reshape(BN * self.Tk, d).contiguous()
        sess = DecodeSession(m, enc_rep, BN, self.Tk, T_max)
        del enc_rep
        sess.t_dev.zero_()
        pl = prompt.tolist()                                     # one host read for the whole prompt
        for t in range(P - 1):                                   # prompt prefill (identical on every row)
            sess.cur.fill_(pl[t])
            sess.step()
            if no_speech is not None and t == no_speech[0]:
                self.ns_prob = self._ns(sess, no_speech[1])
        sess.cur.fill_(pl[P - 1])
        K = max(2, 2) * nb                                       # beams_to_keep: (1 eos token + 1) * k
        top_mask = torch.zeros(K, dtype=torch.bool, device=dev)
        top_mask[:nb] = True
        run_seq = torch.full((B, nb, T_max), self.fill, dtype=torch.int64, device=dev)
        run_seq[:, :, :P] = prompt
        seqs = run_seq.clone()
        run_scores = torch.zeros(B, nb, dtype=torch.float32, device=dev)
        run_scores[:, 1:] = -1e9
        scores = torch.full((B, nb), -1e9, dtype=torch.float32, device=dev)
        finished = torch.zeros(B, nb, dtype=torch.bool, device=dev)
        heur_unsat = torch.ones(B, 1, dtype=torch.bool, device=dev)
        run_bidx = torch.full((B, nb, T_max - P), -1, dtype=torch.int32, device=dev)
        bidx = run_bidx.clone()
        lp, es = self.length_penalty, self.early_stopping
        rows_ident = torch.arange(BN, dtype=torch.int64, device=dev)
        ts = self.ts is not None
        run_last_ts = torch.full((B, nb), -1, dtype=torch.int64, device=dev)     # last timestamp token per beam
        run_sum = torch.zeros(B, nb, dtype=torch.float32, device=dev)            # sum of renormalised log-probs
        fin_sum = torch.zeros(B, nb, dtype=torch.float32, device=dev)
        cur = P
        while True:
            sess.step()                                          # logits of position cur - 1 on every row
            if no_speech is not None and cur == P and no_speech[0] == P - 1:
                self.ns_prob = self._ns(sess, no_speech[1])
            logp = torch.log_softmax(sess.logits[:, :V].float(), dim=-1)
            if self.sup.numel():
                logp[:, self.sup] = -float("inf")
            if cur == P and self.beg.numel():                    # SuppressTokensAtBegin (begin_index = P)
                logp[:, self.beg] = -float("inf")
            if ts:
                logp = self._ts_rules(logp, run_seq, run_last_ts, cur)
            acc = (logp.view(B, nb, V) + run_scores[:, :, None]).reshape(B, nb * V)
            # _get_top_k_continuations
            top_lp, top_i = torch.topk(acc, k=K)
            src = top_i // V
            tok = top_i % V
            if ts:
                # HF's gate sums log_softmax(processed row)[token] along the chosen beam: processed - lse(processed)
                lse = torch.logsumexp(logp, dim=-1).view(B, nb)
                contrib = torch.gather(logp.view(B, nb * V), 1, top_i) - torch.gather(lse, 1, src)
                top_sum = torch.gather(run_sum, 1, src) + contrib
                top_last_ts = torch.where(tok >= self.ts[0], tok, torch.gather(run_last_ts, 1, src))
            top_bidx = self._gather(run_bidx, src)
            top_seq = self._gather(run_seq, src)
            top_seq[:, :, cur] = tok
            top_bidx[:, :, cur - P] = (src + torch.arange(B, device=dev).view(-1, 1) * nb).to(torch.int32)
            # stopping criteria on each candidate: eos, or the sequence reaching max_length
            hits = (tok == self.eos) | (cur + 1 >= T_max)
            # _get_running_beams_for_next_iteration
            run_lp = top_lp + hits.to(torch.float32) * -1.0e9
            nxt = torch.topk(run_lp, k=nb)[1]
            run_seq = self._gather(top_seq, nxt)
            run_scores = self._gather(run_lp, nxt)
            run_bidx = self._gather(top_bidx, nxt)
            if ts:
                run_sum = self._gather(top_sum, nxt)
                run_last_ts = self._gather(top_last_ts, nxt)
            # _update_finished_beams
            just = hits & top_mask[None, :]
            fin_lp = top_lp / ((cur + 1 - P) ** lp)
            full = torch.all(finished, dim=-1, keepdim=True) & (es is True)
            fin_lp = fin_lp + full.to(torch.float32) * -1.0e9
            fin_lp = fin_lp + (~heur_unsat).to(torch.float32) * -1.0e9
            fin_lp = fin_lp + (~just).to(torch.float32) * -1.0e9
            m_seq = torch.cat((seqs, top_seq), 1)
            m_sc = torch.cat((scores, fin_lp), 1)
            m_bi = torch.cat((bidx, top_bidx), 1)
            m_fin = torch.cat((finished, just), 1)
            keep = torch.topk(m_sc, k=nb)[1]
            seqs, scores = self._gather(m_seq, keep), self._gather(m_sc, keep)
            bidx, finished = self._gather(m_bi, keep), self._gather(m_fin, keep)
            if ts:
                fin_sum = self._gather(torch.cat((fin_sum, top_sum), 1), keep)
            # the next step's inputs: each running beam's new token, its source row's caches
            src_rows = run_bidx[:, :, cur - P].reshape(-1).to(torch.int64)
            sess.cur.copy_(run_seq[:, :, cur].reshape(-1))
            cur += 1
            # _check_early_stop_heuristic / _beam_search_has_unfinished_sequences
            if es == "never" and lp > 0.0:
                best_len = T_max - P
            else:
                best_len = cur - P
            best_run = run_scores[:, :1] / (best_len ** lp)
            worst_fin = torch.where(finished, torch.min(scores, dim=1, keepdim=True)[0], torch.full_like(scores, -1e9))
            heur_unsat = heur_unsat & torch.any(best_run > worst_fin, dim=-1, keepdim=True)
            # one host read per step for every decision: continue?  and is the beam reorder the identity (every
            # running beam continues its own row), in which case the cache gather is skipped
            flags = torch.stack([torch.any(heur_unsat), torch.all(finished), torch.all(hits),
                                 (src_rows == rows_ident).all()]).tolist()
            go = flags[0] and not (flags[1] and es is True) and not flags[2]
            if not go or cur >= T_max:
                break
            if not flags[3]:
                for c in sess.self_kv:
                    c[:, :cur - 1].copy_(c[:, :cur - 1].index_select(0, src_rows))
        best = seqs[:, 0]
        gen_len = int(((bidx[:, 0] + 1) != 0).sum(dim=1).max())
        if ts:
            self.sum_logp = fin_sum[:, 0]
        return best[:, P:P + gen_len]


def total_length(cfg, gc, P, max_length=None, max_new_tokens=None):
    """Length cap of prompt + generated tokens, HF _set_max_new_tokens_and_length
    (generation_whisper.py:1919-1945): max_new_tokens counts after the P prompt tokens; a max_length
    (the call's, else generation_config's) is raised by the min(max_target_positions // 2 - 1, P)
    initial tokens; both capped at max_target_positions."""
    if max_new_tokens is not None:
        total = P + int(max_new_tokens)
    else:
        ml = max_length or gc.max_length or cfg.max_target_positions
        total = int(ml) + min(cfg.max_target_positions // 2 - 1, P)
    return min(total, cfg.max_target_positions)


def retrieve_segment(seq, seek_num_frames, ts_begin=50364, input_stride=2):
    """HF `_retrieve_segment` (generation_whisper.py), token part: split a window's tokens at
    consecutive timestamp pairs -> (segments, seek offset in feature frames)."""
    is_ts = [t >= ts_begin for t in seq]
    single_end = is_ts[-2:] == [False, True]
    cut = [i + 1 for i in range(len(seq) - 1) if is_ts[i] and is_ts[i + 1]]
    if not cut:
        return [list(seq)], seek_num_frames
    slices = list(cut)
    if single_end:
        slices.append(len(seq))
    else:
        slices[-1] += 1
    segs, last = [], 0
    for c in slices:
        segs.append(list(seq[last:c]))
        last = c
    off = seek_num_frames if single_end else (seq[last - 2] - ts_begin) * input_stride
    return segs, off


@torch.no_grad()
def generate(model, input_features=None, max_length=None, num_beams=1, return_timestamps=False, language=None,
             task=None, decoder_input_ids=None, max_new_tokens=None, encoder_outputs=None, attention_mask=None,
             use_graph=None, **kw):
    from .config import GenerationConfig
    nb = 1 if num_beams is None else int(num_beams)
    temperature = kw.get("temperature")
    fb = dict(temperature=temperature if temperature is not None else 0.0,
              compression_ratio_threshold=kw.get("compression_ratio_threshold"),
              logprob_threshold=kw.get("logprob_threshold"), no_speech_threshold=kw.get("no_speech_threshold"),
              condition_on_prev_tokens=bool(kw.get("condition_on_prev_tokens") or False), seed=int(kw.get("seed", 0)))
    gc = model.generation_config if model.generation_config is not None else GenerationConfig()
    if not isinstance(gc, GenerationConfig):
        gc = GenerationConfig(gc)
    if gc.eos_token_id is None:
        gc.eos_token_id = model.config.eos_token_id
    cfg = model.config
    use_graph = True if use_graph is None else use_graph
    window = 2 * cfg.max_source_positions                     # 3000 feature frames = 30 s
    # HF (generation_whisper.py:785-898) runs the seek loop for every input when timestamps are predicted, a
    # <= 30 s one included: a window that ends on a timestamp pair before the end of the audio is followed by
    # another window from that timestamp (tests/test_lv2_decode_gpu.py pins it at large-v2 dims)
    seek_loop = bool(return_timestamps) and decoder_input_ids is None
    if encoder_outputs is None and input_features is not None and (input_features.shape[-1] > window or seek_loop):
        return _longform(model, gc, input_features, attention_mask, language, task, max_length, max_new_tokens,
                         use_graph, window, kw.get("_trace"), fallback_batch=bool(kw.get("fallback_batch", True)),
                         num_beams=nb, **fb)
    if kw.get("do_sample") or fb["temperature"] not in (0, 0.0) or fb["logprob_threshold"] is not None \
            or fb["compression_ratio_threshold"] is not None or fb["no_speech_threshold"] is not None:
        # the reference applies fallback / thresholds to long-form inputs only (run_eval.py:659-685)
        raise NotImplementedError("tw generate: temperature fallback and thresholds apply to long-form (> 30 s) "
                                  "inputs, as in the reference; short-form decoding is greedy")
    if encoder_outputs is not None:
        enc = encoder_outputs.last_hidden_state if hasattr(encoder_outputs, "last_hidden_state") else encoder_outputs[0]
        B, Tk = enc.shape[0], enc.shape[1]
        enc16 = enc.reshape(-1, cfg.d_model).to(model.device, model.act_dtype).contiguous()
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
    max_length = total_length(cfg, gc, P, max_length, max_new_tokens)
    if P >= max_length:
        return torch.empty(B, 0, dtype=torch.int64, device=model.device)
    if nb > 1:
        if not bool((prompt == prompt[:1]).all()):
            raise NotImplementedError("tw generate: beam search takes one prompt for every clip")
        return _BeamDecoder(model, gc, B, nb, Tk, P, max_length).run(enc16, prompt[0])
    dec = _Decoder(model, gc, B, Tk, P, max_length, bool(return_timestamps), use_graph)
    if kw.get("_keep") is not None:          # tests: the decoder (and its device caches) outlive the call
        kw["_keep"].append(dec)
    return dec.run(enc16, prompt.to(model.device))


def batch_rows_independent(model):
    """True where each row of a decode batch of <= 8 rows is bit-identical to its batch-1 decode: on the 16-bit
    compute paths every decode-step Linear is a per-row GEMV (d % 256 == 0) or the skinny GEMM, whose K order per
    output does not depend on the batch (no split-K at <= 32 rows); tests/test_fallback_gpu.py runs the skinny
    form (micro, d = 128).  The fp32 path's GEMMs are not shown row-independent, so it decodes one at a time."""
    return model.compute in ("bf16", "fp16")


def row_tokens(raw, eos):
    """One row of a decoded batch as its own batch-1 decode returns it: up to and including its first eos."""
    raw = list(raw)
    return raw[:raw.index(eos) + 1] if eos in raw else raw


def compression_ratio(tokens, vocab_size):
    """HF _retrieve_compression_ratio (generation_whisper.py:1949-1956): raw token bytes (little-endian,
    int(log2(V)/8)+1 bytes each) over their zlib-compressed length."""
    import math
    import zlib
    n = int(math.log2(vocab_size) / 8) + 1
    raw = b"".join(int(t).to_bytes(n, "little") for t in tokens)
    return len(raw) / len(zlib.compress(raw))


def need_fallback(tokens, avg_logprob, no_speech_prob, vocab_size, compression_ratio_threshold=None,
                  logprob_threshold=None, no_speech_threshold=None):
    """HF _need_fallback (generation_whisper.py:1243-1290) -> (needs_fallback, should_skip)."""
    needs, skip = False, False
    if compression_ratio_threshold is not None and compression_ratio(tokens, vocab_size) > compression_ratio_threshold:
        needs = True
    if logprob_threshold is not None and avg_logprob < logprob_threshold:
        needs = True
    if no_speech_threshold is not None and logprob_threshold is not None:
        if avg_logprob < logprob_threshold and no_speech_prob > no_speech_threshold:
            needs, skip = False, True
    return needs, skip


def _bucket(n):
    """Decode-batch size for n rows: the next power of two up to 8 (the GEMV regime: one launch per Linear whatever the
    rows), then the next multiple of 8; the extra rows repeat the first one and are dropped.  A shrinking batch --
    recordings finishing, fewer rows falling back -- then reuses a captured step."""
    if n > 8:
        return (n + 7) // 8 * 8
    b = 1
    while b < n:
        b *= 2
    return b


def _longform_batched(model, gc, feats, lens, init, temps, track, window, trace, max_length, max_new_tokens,
                      compression_ratio_threshold, logprob_threshold, no_speech_threshold, fallback_batch, decoder, trim,
                      seeds_of, ns_token, ts_begin, eos, pad, enc_rows=32):
    """HF's batched sequential long-form (generation_whisper.py:785-898 with generate_with_fallback :970-1117): every
    recording of the call stays in ONE batch window after window -- each seek iteration cuts the current 30 s window
    of every unfinished recording at its own seek (_get_input_segment, zero-padded), encodes them together, decodes
    them together from the same prompt, and a recording whose seek reaches its length leaves the batch
    (_maybe_reduce_batch).  Fallback as generate_with_fallback: the rows whose attempt fails HF's gate are decoded
    again at the next temperature, together; a row is accepted at its first passing attempt (or keeps its last one),
    and a skipped row advances by its window.  run_eval.py:667-681 calls generate on inner_batch_size recordings this
    way; HF's own rows are not batch-invariant either (the encoder and the decoder see the batch), so parity is with
    HF's batched call (tests/test_batched_longform_gpu.py).

    Speculative fallback (fallback_batch, 16-bit paths whose decode rows are independent, batch_rows_independent):
    while the failing rows are few, several temperature levels of them decode as one batch of at most 8 rows (the
    decode step at <= 8 rows is one GEMV launch per Linear, latency-bound: extra rows are nearly free); each row still
    takes its first passing attempt in temperature order, and a row's attempt decodes the same tokens whichever batch
    it sits in (per-row temperature and seed, tw_select_sample_ts), so the result is the level-by-level one."""
    model_cfg = model.config
    dev = model.device
    nmel = feats.shape[1]
    B = feats.shape[0]
    V = model_cfg.vocab_size
    P = len(init)
    ml = total_length(model_cfg, gc, P, max_length, max_new_tokens)
    if P >= ml:
        raise ValueError(f"prompt of {P} tokens leaves no room below max_length {ml}")
    ns = (0, ns_token) if no_speech_threshold is not None else None
    spec = fallback_batch and batch_rows_independent(model)
    seek = [0] * B
    nwin = [0] * B
    outs = [[] for _ in range(B)]
    while True:
        active = [b for b in range(B) if seek[b] < int(lens[b])]          # _maybe_reduce_batch
        if not active:
            break
        nfr = {b: min(window, int(lens[b]) - seek[b]) for b in active}
        # encode the current windows together (chunks of enc_rows bound the encoder's activations)
        enc = {}
        for c0 in range(0, len(active), enc_rows):
            rows = active[c0:c0 + enc_rows]
            segb = torch.zeros(len(rows), nmel, window, dtype=torch.float32, device=dev)
            for i, b in enumerate(rows):
                segb[i, :, :nfr[b]] = feats[b, :, seek[b]:seek[b] + nfr[b]]
            e = model.encode(model.conv_input(segb))
            tk = e.shape[0] // len(rows)
            for i, b in enumerate(rows):
                enc[b] = e[i * tk:(i + 1) * tk]
            del segb
        result = {}                       # b -> (accepted tokens, skip)
        pending = list(active)
        level = 0
        seeds = {b: seeds_of(b, nwin[b]) for b in active}
        while pending and level < len(temps):
            per = max(1, 8 // len(pending)) if spec and level > 0 else 1
            levels = list(range(level, min(len(temps), level + per)))
            attempts = [(b, f) for f in levels for b in pending]
            nb = _bucket(len(attempts))
            pad_n = nb - len(attempts)
            rows_att = attempts + [attempts[0]] * pad_n
            one = len({b for b, _ in rows_att}) == 1
            # the rows' encoder outputs: one window shared by every row (its K/V projected once), else gathered
            e16 = enc[rows_att[0][0]] if one else torch.cat([enc[b] for b, _ in rows_att])
            d_ = decoder(P, ml, nb)
            tl = [temps[f] or 0.0 for _, f in rows_att]
            sl = [seeds[b][f] for b, f in rows_att]
            raws = d_.run(e16, torch.tensor([init] * nb, dtype=torch.int64, device=dev),
                          temperature=tl if nb > 1 else tl[0], seed=sl if nb > 1 else sl[0], no_speech=ns).tolist()
            del e16
            # a batch is cut at its LAST row's first eos: each row is cut at its own first eos, what its own decode
            # returns
            raws = [row_tokens(r, eos) for r in raws[:len(attempts)]]
            decided = set()
            for r, (b, f) in enumerate(attempts):
                if b in decided:
                    continue                                  # accepted at a lower temperature of this batch
                raw = raws[r]
                cand = trim(raw)
                needs, skip = False, False
                if track or compression_ratio_threshold is not None:
                    tg = time.perf_counter()
                    avg = float(d_.sel.sum_logp[r]) / max(len(cand), 1) if track else 0.0
                    nsp = float(torch.exp(d_.ns_logp[r])) if ns is not None else 0.0
                    needs, skip = need_fallback(cand, avg, nsp, V, compression_ratio_threshold, logprob_threshold,
                                                no_speech_threshold)
                    if trace is not None:
                        trace.append(dict(b=b, seek=seek[b], n=nfr[b], T=temps[f], prompt=list(init), raw=list(raw),
                                          avg_logprob=avg, no_speech_prob=nsp, needs_fallback=needs, skip=skip,
                                          batch=nb, gate_ms=(time.perf_counter() - tg) * 1e3))
                elif trace is not None:
                    trace.append(dict(b=b, seek=seek[b], n=nfr[b], T=temps[f], prompt=list(init), raw=list(raw),
                                      batch=nb))
                result[b] = (raw, skip)
                if not needs:
                    decided.add(b)
            pending = [b for b in pending if b not in decided]
            level = levels[-1] + 1
        del enc
        for b in active:
            seq, skip = result[b]
            n = nfr[b]
            nwin[b] += 1
            if skip:
                seek[b] += n
                continue
            if seek[b] + window < int(lens[b]) and seq and seq[-1] == eos:    # not the last window: cut its eos
                seq = seq[:-1]
            if seq and seq[-1] == pad:                                         # trailing pads (pad == eos keeps one)
                k = len(seq)
                while k > 1 and seq[k - 2] == pad:
                    k -= 1
                seq = seq[:k] if pad == eos else seq[:k - 1]
            if not seq:
                seek[b] += n
                continue
            segs, off = retrieve_segment(seq, n, ts_begin)
            for sgm in segs:
                outs[b].extend(sgm)
            seek[b] += off if off > 0 else n          # a closing <|0.00|> pair would not advance: take the window
    L = max((len(o) for o in outs), default=0)
    res = torch.full((B, L), pad, dtype=torch.int64)
    for b, o in enumerate(outs):
        res[b, :len(o)] = torch.tensor(o, dtype=torch.int64)
    return res.to(dev)


def _longform(model, gc, feats, attention_mask, language, task, max_length, max_new_tokens, use_graph, window,
              trace=None, temperature=0.0, compression_ratio_threshold=None, logprob_threshold=None,
              no_speech_threshold=None, condition_on_prev_tokens=False, seed=0, fallback_batch=True, num_beams=1):
    """HF sequential long-form generate (generation_whisper.py step 6): per input, 30 s windows from
    `seek`; each window decoded with timestamp rules at the first temperature of `temperature` and
    re-decoded at the next one while HF's fallback test fails (compression ratio of the token bytes,
    average log-prob of the processed scores, no-speech probability at <|startoftranscript|> -> skip
    the window); trailing eos/pad trimmed, segments split at consecutive timestamps, seek advanced
    by the last timestamp (or the whole window on a single-timestamp ending).  With
    condition_on_prev_tokens (and the accepted temperature < 0.5) the next window's prompt is
    <|startofprev|> + the last max_target_positions // 2 - 1 tokens of the clip's segments (a
    segment's closing timestamp of a double-timestamp ending dropped) + the task prompt.  Returns
    the concatenated segment tokens, right-padded with pad.  Sampled windows draw from
    softmax(x / T) with the engine's counter-based RNG (seeded by `seed`, the clip, the window and
    the fallback index), not torch's RNG stream.  Once a window's first attempt fails, the remaining
    temperatures are decoded together as one batch (fallback_batch; identical tokens and gates to decoding
    them one by one, see the loop below).  num_beams > 1 (run_eval.py --num_beams with timestamps / long-form): as HF
    generate_with_fallback, a temperature-0 attempt is a beam search over the window (_BeamDecoder with the timestamp
    rules; its gates from the chosen hypothesis's per-step processed scores), a sampled attempt keeps one beam."""
    cfg = model.config
    dev = model.device
    feats = feats.to(dev, torch.float32)
    B, nmel, T = feats.shape
    lens = attention_mask.sum(-1).tolist() if attention_mask is not None else [T] * B
    init = build_prompt(gc, language, task, True)
    temps = tuple(temperature) if isinstance(temperature, (list, tuple)) else (temperature,)
    track = (logprob_threshold is not None or no_speech_threshold is not None or any(t and t > 0 for t in temps)
             or len(temps) > 1)
    eos, pad = int(gc.eos_token_id), int(gc.pad_token_id if gc.pad_token_id is not None else gc.eos_token_id)
    ts_begin = int(gc.no_timestamps_token_id) + 1
    ns_token = int(gc.no_timestamps_token_id) - 1
    V = cfg.vocab_size
    cut_off = cfg.max_target_positions // 2 - 1
    prev_sot = gc.get("prev_sot_token_id") if hasattr(gc, "get") else None
    if prev_sot is None:
        sup = list(gc.suppress_tokens or [])
        prev_sot = sup[-2] if len(sup) >= 2 else None
    decoders = {}

    def decoder(P, ml, nb=1):
        key = (P, ml, nb)
        if key in decoders:
            decoders[key] = decoders.pop(key)            # most recently used last
        else:
            # each decoder holds a captured step and the cross-attention K/V of its rows (246 MB per row at
            # large-v2): keep the three most recently used
            while len(decoders) >= 3:
                decoders.pop(next(iter(decoders)))
            decoders[key] = _Decoder(model, gc, nb, cfg.max_source_positions, P, ml, True, use_graph, track)
        return decoders[key]

    def trim(raw):
        cand = list(raw)
        if cand and cand[-1] == pad:                     # HF: padding removed except one eos
            k = len(cand)
            while k > 1 and cand[k - 2] == pad:
                k -= 1
            cand = cand[:k] if pad == eos else cand[:k - 1]
        return cand

    def seeds_of(b, nwin):
        return [(seed * 1000003 + b * 7919 + nwin * 131 + fi) & ((1 << 63) - 1) for fi in range(len(temps))]

    nbeam = max(1, int(num_beams or 1))
    beam_ts = (ts_begin, int(gc.no_timestamps_token_id), gc.max_initial_timestamp_index
               if "max_initial_timestamp_index" in gc else None)
    if nbeam == 1 and not condition_on_prev_tokens:
        return _longform_batched(model, gc, feats, lens, init, temps, track, window, trace, max_length,
                                 max_new_tokens, compression_ratio_threshold, logprob_threshold, no_speech_threshold,
                                 fallback_batch, decoder, trim, seeds_of, ns_token, ts_begin, eos, pad)
    # conditioning on the previous windows' text (per-recording prompts of different lengths: HF left-pads them under
    # a decoder attention mask) and beam search: one recording at a time
    seg_in = torch.zeros(1, nmel, window, dtype=torch.float32, device=dev)
    outs = []
    for b in range(B):
        Tb = int(lens[b])
        seek, out, segments, nwin = 0, [], [], 0
        cond = bool(condition_on_prev_tokens)
        while seek < Tb:
            n = min(window, Tb - seek)
            seg_in.zero_()
            seg_in[0, :, :n] = feats[b, :, seek:seek + n]
            enc16 = model.encode(model.conv_input(seg_in))
            prompt = list(init)
            if cond and segments and prev_sot is not None:
                prev = []
                for st in segments:
                    prev.extend(st[:-1] if len(st) > 2 and st[-2] >= ts_begin else st)
                prompt = [int(prev_sot)] + prev[-cut_off:] + init
            P = len(prompt)
            ml = total_length(cfg, gc, P, max_length, max_new_tokens)
            if P >= ml:
                raise ValueError(f"prompt of {P} tokens leaves no room below max_length {ml}")
            dec = decoder(P, ml)
            ptens = torch.tensor([prompt], dtype=torch.int64, device=dev)
            ns = (P - len(init), ns_token) if no_speech_threshold is not None else None
            skip, t_acc, seq = False, temps[0], []
            # attempt fi draws with seed(fi); attempts 1.. run as ONE batch (one row per remaining temperature,
            # speculatively) once attempt 0 fails its gate: a batch-1 decode step is launch-bound, so the
            # batch costs about what one attempt does.  Rows are independent (per-row temperature / seed,
            # tw_select_sample_ts), so each row decodes exactly the tokens its sequential attempt would, and the
            # first passing row in temperature order is accepted, as HF generate_with_fallback accepts it.
            seeds = seeds_of(b, nwin)
            attempts = [(0, dec, enc16, ptens, [temps[0] or 0.0], [seeds[0]])]
            rest = list(range(1, len(temps)))
            # fallback_batch=False: one attempt at a time (A/B, tests); so does the fp32 compute path, whose rows are
            # not shown independent of the batch (batch_rows_independent), and a beam search at temperature 0 later
            # in the schedule
            per = 8 if fallback_batch and batch_rows_independent(model) else 1
            if nbeam > 1 and any(not temps[f] for f in rest):
                per = 1
            for fb in range(0, len(rest), per):
                grp = rest[fb:fb + per]
                attempts.append((grp[0], None, None, None, [temps[f] or 0.0 for f in grp], [seeds[f] for f in grp]))
            for fi0, d_, e_, p_, tl, sl in attempts:
                if nbeam > 1 and len(tl) == 1 and not tl[0]:   # temperature 0 with num_beams: the beam search
                    bd = _BeamDecoder(model, gc, 1, nbeam, cfg.max_source_positions, P, ml, timestamps=beam_ts)
                    raw = row_tokens(bd.run(enc16, prompt, no_speech=ns)[0].tolist(), eos)
                    avg = float(bd.sum_logp[0]) / max(len(trim(raw)), 1)
                    nsp = float(bd.ns_prob[0]) if ns is not None else 0.0
                    raws, gates, nbatch = [raw], [(avg, nsp)], 1
                else:
                    if d_ is None:                           # a speculative batch of the remaining attempts
                        nb = len(tl)
                        d_ = decoder(P, ml, nb)
                        e_ = enc16                           # shared by the rows (DecodeSession.set_encoder)
                        p_ = ptens.repeat(nb, 1)
                    raws = d_.run(e_, p_, temperature=tl if len(tl) > 1 else tl[0],
                                  seed=sl if len(sl) > 1 else sl[0], no_speech=ns).tolist()
                    # a batch is cut at its LAST row's first eos, so a row that finished earlier carries extra eos
                    # (=pad) columns; each row is cut at its own first eos, which is what its batch-1 decode returns
                    raws = [row_tokens(r, eos) for r in raws]
                    gates, nbatch = None, len(raws)
                done_here = False
                for r, raw in enumerate(raws):
                    fi, temp = fi0 + r, temps[fi0 + r]
                    cand = trim(raw)
                    needs = False
                    if track or compression_ratio_threshold is not None or (nbeam > 1 and gates is not None):
                        tg = time.perf_counter()      # gate cost: log-prob / no-speech readback + compression ratio
                        if gates is not None:
                            avg, nsp = gates[r]
                        else:
                            avg = float(d_.sel.sum_logp[r]) / max(len(cand), 1) if track else 0.0
                            nsp = float(torch.exp(d_.ns_logp[r])) if ns is not None else 0.0
                        needs, skip = need_fallback(cand, avg, nsp, V, compression_ratio_threshold, logprob_threshold,
                                                    no_speech_threshold)
                        if trace is not None:
                            trace.append(dict(b=b, seek=seek, n=n, T=temp, prompt=list(prompt), raw=list(raw),
                                              avg_logprob=avg, no_speech_prob=nsp, needs_fallback=needs, skip=skip,
                                              batch=nbatch, gate_ms=(time.perf_counter() - tg) * 1e3))
                    elif trace is not None:
                        trace.append(dict(b=b, seek=seek, n=n, T=temp, prompt=list(prompt), raw=list(raw),
                                          batch=nbatch))
                    seq, t_acc = raw, temp
                    if not needs:
                        done_here = True
                        break
                if done_here:
                    break
            nwin += 1
            cond = bool(condition_on_prev_tokens) and (t_acc is None or t_acc < 0.5)
            if skip:
                seek += n
                continue
            if seek + window < Tb and seq and seq[-1] == eos:   # not the last window: cut a predicted eos
                seq = seq[:-1]
            if seq and seq[-1] == pad:                          # trailing pads (pad == eos keeps one)
                k = len(seq)
                while k > 1 and seq[k - 2] == pad:
                    k -= 1
                seq = seq[:k] if pad == eos else seq[:k - 1]
            if not seq:
                seek += n
                continue
            segs, off = retrieve_segment(seq, n, ts_begin)
            for sgm in segs:
                out.extend(sgm)
                segments.append(list(sgm))
            seek += off if off > 0 else n          # a closing <|0.00|> pair would not advance: take the window
        outs.append(out)
    L = max((len(o) for o in outs), default=0)
    res = torch.full((B, L), pad, dtype=torch.int64)
    for b, o in enumerate(outs):
        res[b, :len(o)] = torch.tensor(o, dtype=torch.int64)
    return res.to(dev)
