"""Label side of the step (host, integer work) and synthetic inputs.

  prepare_labels   training/run_distillation.py:1221-1274 (prepare_train_dataset text targets,
                   on token ids: timestamp filtering w.p. 1 - timestamp_probability with
                   <|notimestamps|> inserted at position 3 (multilingual), <|startofprev|>
                   prompt w.p. condition_on_prev_probability, cut-offs 224 / 448)
  DataCollatorSpeechSeq2SeqWithPadding
                   :437-511 (pad labels to max_length with pad 50257, split into
                   decoder_input_ids / labels, -100 on padding and on the prompt incl. SOT)
  synthetic_*      SURVEY.md §8(d) benchmark inputs (30 s 16 kHz sines + noise; labels of
                   length U[32, 440] with 20 % prompts).
"""
from __future__ import annotations

import math

import numpy as np
import torch

EOT = PAD = 50257
SOT, ZH, TRANSCRIBE, STARTOFPREV, NOTIMESTAMPS = 50258, 50260, 50359, 50361, 50363
TIMESTAMP_BEGIN = NOTIMESTAMPS   # tokenizer.all_special_ids[-1] (:1129)
WHITESPACE = 220


def prepare_labels(token_ids_batch, prev_batch, rng, timestamp_probability=0.5, condition_on_prev_probability=0.2,
                   max_label_length=448, is_multilingual=True, has_prev_column=True):
    timestamp_position = 3 if is_multilingual else 1
    cutoff = max_label_length // 2
    out, unprompted = [], []
    prev_ids = None
    for prev_in, token_ids in zip(prev_batch, token_ids_batch):
        token_ids = list(token_ids)
        if prev_in is not None:
            prev_ids = list(prev_in)
        has_ts = any(t > TIMESTAMP_BEGIN for t in token_ids)
        predict_ts = True
        if has_ts:
            predict_ts = bool(rng.binomial(1, timestamp_probability))
            if not predict_ts:
                token_ids = [t for t in token_ids if t < TIMESTAMP_BEGIN]
                token_ids.insert(timestamp_position, TIMESTAMP_BEGIN)
        unprompted.append(token_ids)
        cond = bool(rng.binomial(1, condition_on_prev_probability))
        if not cond:
            prev_ids = None
        elif not has_prev_column and len(unprompted) > 1:
            prev_ids = unprompted[-2]
        if prev_ids is not None:
            if has_ts and not predict_ts:
                prev_ids = [t if t < TIMESTAMP_BEGIN else WHITESPACE for t in prev_ids]
            if len(prev_ids) > cutoff:
                prev_ids = [STARTOFPREV] + prev_ids[-cutoff + 1:]
            if len(prev_ids + token_ids) > max_label_length:
                trim = len(prev_ids + token_ids) - max_label_length + 1
                prev_ids = [STARTOFPREV] + prev_ids[trim:]
            token_ids = prev_ids + token_ids
        out.append(token_ids)
    return out


class DataCollatorSpeechSeq2SeqWithPadding:
    def __init__(self, processor=None, decoder_start_token_id=SOT, decoder_prev_token_id=STARTOFPREV,
                 input_padding="longest", target_padding="max_length", max_target_length=448, pad_token_id=PAD):
        self.processor = processor
        self.decoder_start_token_id = decoder_start_token_id
        self.decoder_prev_token_id = decoder_prev_token_id
        self.max_target_length = max_target_length
        self.pad_token_id = pad_token_id

    def collate_labels(self, label_lists):
        L = max(self.max_target_length, max(len(x) for x in label_lists))
        B = len(label_lists)
        ids = np.full((B, L), self.pad_token_id, dtype=np.int64)
        att = np.zeros((B, L), dtype=np.int64)
        for i, x in enumerate(label_lists):
            ids[i, : len(x)] = x
            att[i, : len(x)] = 1
        dec = ids[:, :-1].copy()
        lab = ids[:, 1:].copy()
        lab[att[:, 1:] != 1] = -100
        bos = np.argmax(lab == self.decoder_start_token_id, axis=1)
        bos = np.where(bos > 0, bos + 1, bos)
        lab = np.where(np.arange(lab.shape[1])[None, :] < bos[:, None], -100, lab)
        return torch.from_numpy(dec), torch.from_numpy(lab)

    def __call__(self, features):
        dec, lab = self.collate_labels([f["labels"] for f in features])
        feats = [f["input_features"] for f in features]
        batch = {"input_features": torch.stack([torch.as_tensor(x) for x in feats])}
        batch["labels"], batch["decoder_input_ids"] = lab, dec
        return batch


def synthetic_label_lists(B, seed=0, prompt_fraction=0.2, min_len=32, max_len=440, lang=ZH):
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for _ in range(B):
        n = int(rng.integers(min_len, max_len + 1))
        body = rng.integers(0, EOT, size=max(n - 5, 1)).tolist()
        seq = [SOT, lang, TRANSCRIBE, NOTIMESTAMPS] + body + [EOT]
        if rng.random() < prompt_fraction:
            p = int(rng.integers(16, 65))
            prompt = [STARTOFPREV] + rng.integers(0, EOT, size=p).tolist()
            room = 448 - len(seq)
            if room > 1:
                seq = prompt[:room] + seq
        out.append(seq[:448])
    return out


def synthetic_audio(B, seed=0, seconds=30.0, device="cuda", length=480000):
    """x_i(t) = 0.5 sin(2π(220 + 37 i) t) + 0.01 N(0,1) as a [B, length] fp32 device tensor (zero-padded /
    truncated to `length` samples: 480 000 = the 30 s window; pass length=None for the clip's own
    length, e.g. a long-form input)."""
    n = int(seconds * 16000)
    length = n if length is None else length
    t = torch.arange(n, device=device, dtype=torch.float64) / 16000.0
    g = torch.Generator(device=device).manual_seed(1234 + seed)
    f = 220.0 + 37.0 * torch.arange(B, device=device, dtype=torch.float64)[:, None]
    x = 0.5 * torch.sin(2 * math.pi * f * t[None, :]) + 0.01 * torch.randn(B, n, generator=g, device=device,
                                                                           dtype=torch.float64)
    out = torch.zeros(B, length, dtype=torch.float32, device=device)
    k = min(n, length)
    out[:, :k] = x[:, :k].float()
    return out
