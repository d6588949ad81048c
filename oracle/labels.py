"""ORACLE (test infrastructure only): restatement of the label side of the step.

* `prepare_labels` restates `prepare_train_dataset`'s text-target logic,
  `training/run_distillation.py:1221-1274`, on token ids (the tokenizer vocab is not
  available offline): timestamp filtering with probability
  1 - timestamp_probability (`:1234-1242`, `<|notimestamps|>` = timestamp_begin
  inserted at position 3 for multilingual), `<|startofprev|>` prompt with
  probability condition_on_prev_probability (`:1244-1269`, cut-offs 224 / 448).
  Random draws use `rng.binomial(1, p)` in the same order as the reference's
  `np.random.binomial` calls (pass np.random.RandomState(seed) to match a seeded
  global numpy stream).
* `collate` restates `DataCollatorSpeechSeq2SeqWithPadding.__call__`,
  `training/run_distillation.py:471-511`, with `tokenizer.pad(max_length=448,
  padding="max_length")` right-padding with pad_token_id 50257.
* `shift_tokens_right` restates HF:modeling_whisper.py:68-81 (the teacher's
  decoder input when only `labels` are passed, `run_distillation.py:1534`).
"""
from __future__ import annotations

import numpy as np

from .weights import SPECIAL

TIMESTAMP_BEGIN = SPECIAL["notimestamps"]  # tokenizer.all_special_ids[-1]  (:1129)
DECODER_PREV = SPECIAL["startofprev"]      # tokenizer.all_special_ids[-3]  (:1133)
WHITESPACE = 220                            # (:1134)


def prepare_labels(token_ids_batch, prev_batch, rng, timestamp_probability=0.5,
                   condition_on_prev_probability=0.2, max_label_length=448,
                   is_multilingual=True, has_prev_column=True):
    """token_ids_batch: list of token-id lists (already with special tokens).
    prev_batch: list of previous-segment token-id lists or None (cool_dataset's
    `condition_on_prev`).  Returns list of label token-id lists."""
    timestamp_position = 3 if is_multilingual else 1
    prompt_cutoff_length = max_label_length // 2
    all_token_ids, all_unprompted = [], []
    prev_ids = None
    for prev_in, token_ids in zip(prev_batch, token_ids_batch):
        token_ids = list(token_ids)
        if prev_in is not None:
            prev_ids = list(prev_in)
        has_timestamps = any(t > TIMESTAMP_BEGIN for t in token_ids)
        predict_timestamps = True
        if has_timestamps:
            predict_timestamps = bool(rng.binomial(1, timestamp_probability))
            if not predict_timestamps:
                token_ids = [t for t in token_ids if t < TIMESTAMP_BEGIN]
                token_ids.insert(timestamp_position, TIMESTAMP_BEGIN)
        all_unprompted.append(token_ids)
        condition_on_prev = bool(rng.binomial(1, condition_on_prev_probability))
        if not condition_on_prev:
            prev_ids = None
        elif not has_prev_column and len(all_unprompted) > 1:
            prev_ids = all_unprompted[-2]
        if prev_ids is not None:
            if has_timestamps and not predict_timestamps:
                prev_ids = [t if t < TIMESTAMP_BEGIN else WHITESPACE for t in prev_ids]
            if len(prev_ids) > prompt_cutoff_length:
                prev_ids = prev_ids[-prompt_cutoff_length + 1:]
                prev_ids = [DECODER_PREV] + prev_ids
            if len(prev_ids + token_ids) > max_label_length:
                trim = len(prev_ids + token_ids) - max_label_length + 1
                prev_ids = prev_ids[trim:]
                prev_ids = [DECODER_PREV] + prev_ids
            token_ids = prev_ids + token_ids
        all_token_ids.append(token_ids)
    return all_token_ids


def collate(label_lists, decoder_start_token_id=SPECIAL["sot"], pad_token_id=SPECIAL["pad"],
            max_target_length=448):
    """-> (decoder_input_ids int64[B, L-1], labels int64[B, L-1]) with L = max_target_length
    (or the longest sequence if longer, as tokenizer.pad does not truncate)."""
    L = max(max_target_length, max(len(x) for x in label_lists))
    B = len(label_lists)
    ids = np.full((B, L), pad_token_id, dtype=np.int64)
    att = np.zeros((B, L), dtype=np.int64)
    for i, x in enumerate(label_lists):
        ids[i, : len(x)] = x
        att[i, : len(x)] = 1
    decoder_input_ids = ids[:, :-1].copy()
    labels = ids[:, 1:].copy()
    labels[att[:, 1:] != 1] = -100
    bos_index = np.argmax(labels == decoder_start_token_id, axis=1)
    bos_index = np.where(bos_index > 0, bos_index + 1, bos_index)
    prompt_mask = np.arange(labels.shape[1])[None, :] < bos_index[:, None]
    labels = np.where(prompt_mask, -100, labels)
    return decoder_input_ids, labels


def shift_tokens_right(labels, pad_token_id=SPECIAL["pad"], decoder_start_token_id=SPECIAL["sot"]):
    labels = np.asarray(labels)
    out = np.zeros_like(labels)
    out[:, 1:] = labels[:, :-1]
    out[:, 0] = decoder_start_token_id
    out[out == -100] = pad_token_id
    return out


def synthetic_label_lists(B, seed=0, prompt_fraction=0.2, min_len=32, max_len=440,
                          lang=SPECIAL["zh"]):
    """SURVEY.md §8(d) synthetic labels: length U[32,440]; prefix
    [SOT, zh, transcribe, notimestamps]; body U[0, 50257); EOT; 20% of clips carry a
    <|startofprev|> prompt of 16-64 tokens (kept within 448)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for _ in range(B):
        n = int(rng.integers(min_len, max_len + 1))
        body = rng.integers(0, SPECIAL["eot"], size=max(n - 5, 1)).tolist()
        seq = [SPECIAL["sot"], lang, SPECIAL["transcribe"], SPECIAL["notimestamps"]] + body + [SPECIAL["eot"]]
        if rng.random() < prompt_fraction:
            p = int(rng.integers(16, 65))
            prompt = [SPECIAL["startofprev"]] + rng.integers(0, SPECIAL["eot"], size=p).tolist()
            room = 448 - len(seq)
            if room > 1:
                seq = prompt[: room] + seq
        out.append(seq[:448])
    return out
