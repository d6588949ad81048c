"""ORACLE (test infrastructure only): greedy decode restatement.

Reference decode calls: `training/run_distillation.py:1580-1584` (generate_step),
`training/run_pseudo_labelling.py:917-922` (`generate(num_beams=1, language, task)`),
`pseudo-labelling/initial_inference.py:36-41` (faster-whisper; unpinned and absent,
SURVEY.md finding 10 -> parity pinned to HF greedy generate).

HF Whisper generate (HF:generation_whisper.py) with language/task and no timestamps:
prompt [SOT, lang, task, <|notimestamps|>]; per step logits of the last position,
SuppressTokens (generation_config.suppress_tokens) every step, SuppressTokensAtBegin
([220, eos]) at the first generated step (HF:generation/logits_process.py), argmax,
stop at eos or max_length.  This oracle recomputes the whole prefix each step (no
cache) so it shares nothing with the KV-cache path it checks.

Timestamps (`return_timestamps=True`): HF WhisperTimeStampLogitsProcessor (transformers
logits_process.py; applied after SuppressTokensAtBegin and SuppressTokens, generation_whisper.py
`_retrieve_logit_processors`) restated in `timestamp_rules`.  Long-form (input longer than 3000
frames, run_eval.py:659-685 -> HF generate): the sequential window loop of generation_whisper.py
(`generate` step 6, `_retrieve_segment`, the eos/pad trimming of `generate_with_fallback`) with
temperature 0, restated in `longform`, together with the deterministic part of temperature
fallback (generation_whisper.py `generate_with_fallback` :970-1090, `_need_fallback` :1243-1290,
`_retrieve_avg_logprobs` :1958-1975, `_retrieve_compression_ratio` :1949-1956,
WhisperNoSpeechDetection logits_process.py:2050-2112) and previous-text conditioning
(`_prepare_decoder_input_ids` :1853-1905 with `_pad_to_max_length`'s skip_ending_double_timestamps):
the oracle decodes the temperature-0 attempt only, so it pins the fallback decisions, the
skipped windows, the average log-probs / no-speech probabilities and the conditioned prompts,
not the sampled retries (those draw from a different RNG by design).
"""
from __future__ import annotations

import torch

from .whisper_ref import Ref


def greedy(model: Ref, feats, prompt, max_length=448, suppress_tokens=(), begin_suppress=(220, 50257),
           eos=50257, return_scores=False):
    enc = model.encoder(feats)
    B = feats.shape[0]
    ids = torch.tensor(prompt, dtype=torch.long).unsqueeze(0).repeat(B, 1)
    done = torch.zeros(B, dtype=torch.bool)
    scores = []
    while ids.shape[1] < max_length:
        h = model.decoder(ids, enc)
        lg = model.logits(h[:, -1:])[:, 0].clone()
        if len(suppress_tokens):
            lg[:, list(suppress_tokens)] = float("-inf")
        if ids.shape[1] == len(prompt) and len(begin_suppress):
            lg[:, list(begin_suppress)] = float("-inf")
        scores.append(lg)
        nxt = lg.argmax(-1)
        nxt = torch.where(done, torch.full_like(nxt, eos), nxt)
        ids = torch.cat([ids, nxt[:, None]], 1)
        done |= nxt == eos
        if bool(done.all()):
            break
    return (ids, scores) if return_scores else ids


TS_BEGIN, NO_TS = 50364, 50363


def timestamp_rules(lg, gen, first, ts_begin=TS_BEGIN, no_ts=NO_TS, eos=50257, max_initial=None, apply_mass=True):
    """HF WhisperTimeStampLogitsProcessor on one row.  lg: fp32 [V] scores after the suppress
    processors, gen: tokens generated so far in this window (after the prompt).  apply_mass=False
    skips the final "timestamp probability mass beats every text token" step (tests use it to
    accept either branch when that comparison is within rounding noise)."""
    lg = lg.clone()
    lg[no_ts] = float("-inf")
    last_ts = len(gen) >= 1 and gen[-1] >= ts_begin
    pen_ts = len(gen) < 2 or gen[-2] >= ts_begin
    if last_ts:
        if pen_ts:
            lg[ts_begin:] = float("-inf")
        else:
            lg[:eos] = float("-inf")
    stamps = [t for t in gen if t >= ts_begin]
    if stamps:
        lim = stamps[-1] if (last_ts and not pen_ts) else stamps[-1] + 1
        lg[ts_begin:lim] = float("-inf")
    if first:
        lg[:ts_begin] = float("-inf")
        if max_initial is not None:
            lg[ts_begin + max_initial + 1:] = float("-inf")
    if not apply_mass:
        return lg
    lp = torch.log_softmax(lg.float(), -1)
    if lp[ts_begin:].logsumexp(-1) > lp[:ts_begin].max():
        lg[:ts_begin] = float("-inf")
    return lg


def greedy_ts(model: Ref, feats, prompt, max_length=448, suppress_tokens=(), begin_suppress=(220, 50257),
              eos=50257, max_initial=None, enc=None, stats=None, sot_pos=None, no_speech_token=50362):
    """Greedy decode of one 3000-frame window with the timestamp rules (no cache).  stats (a dict,
    batch of one): 'scores' = the processed score rows of every step, 'no_speech_prob' =
    softmax(raw logits at position sot_pos)[no_speech_token]."""
    enc = model.encoder(feats) if enc is None else enc
    B = enc.shape[0]
    ids = torch.tensor(prompt, dtype=torch.long).unsqueeze(0).repeat(B, 1)
    done = torch.zeros(B, dtype=torch.bool)
    if stats is not None:
        stats["scores"] = []
    while ids.shape[1] < max_length:
        h = model.decoder(ids, enc)
        if stats is not None and sot_pos is not None and ids.shape[1] == len(prompt):
            raw = model.logits(h[:, sot_pos:sot_pos + 1])[0, 0].float()
            stats["no_speech_prob"] = float(torch.softmax(raw, -1)[no_speech_token])
        lg = model.logits(h[:, -1:])[:, 0].float().clone()
        if len(suppress_tokens):
            lg[:, list(suppress_tokens)] = float("-inf")
        first = ids.shape[1] == len(prompt)
        if first and len(begin_suppress):
            lg[:, list(begin_suppress)] = float("-inf")
        nxt = torch.empty(B, dtype=torch.long)
        for b in range(B):
            row = timestamp_rules(lg[b], ids[b, len(prompt):].tolist(), first, eos=eos, max_initial=max_initial)
            nxt[b] = row.argmax()
            if stats is not None and b == 0:
                stats["scores"].append(row)
        nxt = torch.where(done, torch.full_like(nxt, eos), nxt)
        ids = torch.cat([ids, nxt[:, None]], 1)
        done |= nxt == eos
        if bool(done.all()):
            break
    return ids


def retrieve_segment(seq, seek_num_frames, ts_begin=TS_BEGIN, input_stride=2):
    """HF `_retrieve_segment` (token part): -> (list of token lists, seek offset in frames)."""
    is_ts = [t >= ts_begin for t in seq]
    single_end = is_ts[-2:] == [False, True]
    cut = [i + 1 for i in range(len(seq) - 1) if is_ts[i] and is_ts[i + 1]]
    if cut:
        slices = list(cut)
        if single_end:
            slices.append(len(seq))
        else:
            slices[-1] += 1
        segs, last = [], 0
        for c in slices:
            segs.append(seq[last:c])
            last = c
        if single_end:
            off = seek_num_frames
        else:
            off = (seq[last - 2] - ts_begin) * input_stride
        return segs, off
    return [list(seq)], seek_num_frames


def compression_ratio(tokens, vocab_size=51865):
    import math
    import zlib
    n = int(math.log2(vocab_size) / 8) + 1
    raw = b"".join(int(t).to_bytes(n, "little") for t in tokens)
    return len(raw) / len(zlib.compress(raw))


def avg_logprob(scores, tokens):
    """_retrieve_avg_logprobs at temperature 0: scores cut to the token count, log_softmax, sum of the
    chosen tokens' log-probs / len(tokens)."""
    sc = torch.stack(scores)[:len(tokens)]
    toks = tokens[-sc.shape[0]:]
    lp = torch.log_softmax(sc.float(), -1)
    return float(sum(lp[i, toks[i]] for i in range(lp.shape[0])) / len(toks))


def longform(model: Ref, feats_long, prompt, suppress_tokens=(), begin_suppress=(220, 50257), eos=50257,
             max_length=448, max_initial=None, window=3000, condition_on_prev_tokens=False, prev_sot=50361,
             logprob_threshold=None, no_speech_threshold=None, compression_ratio_threshold=None, trace=None,
             max_target_positions=448, vocab_size=51865):
    """HF sequential long-form generate at temperature 0 for ONE input [80, T]: returns the
    concatenated segment tokens.  Thresholds: a window whose fallback test fails is kept as decoded
    (no further temperature here); a window HF would skip (avg log-prob below logprob_threshold and
    no-speech probability above no_speech_threshold) contributes nothing and seek moves a window.
    trace: per-window dicts {seek, prompt, tokens, avg_logprob, no_speech_prob, needs_fallback, skip}."""
    T = feats_long.shape[-1]
    seek, out, segments = 0, [], []
    cut_off = max_target_positions // 2 - 1
    ts_begin = TS_BEGIN
    while seek < T:
        n = min(window, T - seek)
        seg = torch.zeros(1, feats_long.shape[0], window, dtype=feats_long.dtype)
        seg[0, :, :n] = feats_long[:, seek:seek + n]
        pr = list(prompt)
        if condition_on_prev_tokens and segments:
            prev = []
            for st in segments:
                prev.extend(st[:-1] if len(st) > 2 and st[-2] >= ts_begin else st)
            pr = [prev_sot] + prev[-cut_off:] + list(prompt)
        stats = {}
        ids = greedy_ts(model, seg, pr, max_length=max_length, suppress_tokens=suppress_tokens,
                        begin_suppress=begin_suppress, eos=eos, max_initial=max_initial, stats=stats,
                        sot_pos=len(pr) - len(prompt))
        seq = ids[0, len(pr):].tolist()
        cand = list(seq)
        if cand and cand[-1] == eos:               # padding removed except one eos (pad == eos)
            k = len(cand)
            while k > 1 and cand[k - 2] == eos:
                k -= 1
            cand = cand[:k]
        avg = avg_logprob(stats["scores"], cand) if cand else 0.0
        nsp = stats.get("no_speech_prob", 0.0)
        needs, skip = False, False
        if compression_ratio_threshold is not None and compression_ratio(cand, vocab_size) > compression_ratio_threshold:
            needs = True
        if logprob_threshold is not None and avg < logprob_threshold:
            needs = True
        if no_speech_threshold is not None and logprob_threshold is not None and avg < logprob_threshold \
                and nsp > no_speech_threshold:
            needs, skip = False, True
        if trace is not None:
            trace.append(dict(seek=seek, prompt=pr, tokens=cand, avg_logprob=avg, no_speech_prob=nsp,
                              needs_fallback=needs, skip=skip))
        if skip:
            seek += n
            continue
        not_final = seek + window < T
        if not_final and seq and seq[-1] == eos:
            seq = seq[:-1]
        if seq and seq[-1] == eos:                 # pad == eos: keep one eos (HF keeps it)
            k = len(seq)
            while k > 1 and seq[k - 2] == eos:
                k -= 1
            seq = seq[:k]
        if not seq:
            seek += n
            continue
        segs, off = retrieve_segment(seq, n)
        for sgm in segs:
            out.extend(sgm)
            segments.append(list(sgm))
        seek += off if off > 0 else n
    return out
