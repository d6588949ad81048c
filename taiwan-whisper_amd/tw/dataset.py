"""Training data feed: the NTU-COOL manifest dataset, per-rank sharding and a
prefetching feed whose log-mel runs on the GPU kernel.

Reference behaviour restated here:
  load_audio_fpaths        dataset/cool_dataset.py:94-104   (manifest: first line = root unless a
                                                             root is given, then one relative path per line)
  read_transcript          dataset/cool_dataset.py:63-83    (the 5-line .txt next to each .flac:
                                                             line 0 whisper transcript, line 2 last-segment
                                                             transcript, line 4 previous transcript)
  trim_last_segment        dataset/cool_dataset.py:20-31    (cut transcript + audio at the last timestamp)
  append_last_segment      dataset/cool_dataset.py:33-47    (the reference function returns None: its
                                                             handler table makes it unusable; restated with
                                                             the evident intent, returning the feature)
  WhisperTokenizerAdapter  training/run_distillation.py:996-1007, 1081, 1229-1231 (WhisperTokenizerFast with
                           the 1501 added timestamp tokens and prefix tokens [SOT, lang, task]; special
                           tokens are atomic, text goes to the BPE)
  prepare_train_batch      training/run_distillation.py:1207-1274 (prepare_train_dataset) + the collator
  shard_micro_batches      accelerate's batch dispatcher over the streaming dataset
                           (run_distillation.py:1645-1652): rank r of N consumes global micro-batch
                           k*N + r; an incomplete final group is completed from the start of the stream
                           (accelerate even_batches), so every rank steps the same number of times.
Differences by design: each rank reads only its own clips (no rank-0 read + broadcast of 491 MB per
step); log-mel runs on the GPU (tw_logmel) instead of CPU dataloader workers; host work
(audio decode, tokenization, label sampling) runs in a thread pool ahead of the step.

Audio decoding: soundfile (libsndfile) when importable, as the reference; without it (this image) FLAC
through the native decoder in libtw_hip.so (tw_flac_decode, host code: csrc/flac.cpp), WAV (PCM
8/16/24/32-bit) via the standard library and .npy arrays; samples as soundfile returns them (float64,
integer PCM / 2^(bits-1)).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import os.path as osp
import re
import wave
from typing import Callable, Iterable, List, Optional, Sequence

import numpy as np
import torch

from .data import (EOT, NOTIMESTAMPS, SOT, STARTOFPREV, TRANSCRIBE, DataCollatorSpeechSeq2SeqWithPadding,
                   prepare_labels)

SAMPLING_RATE = 16000
_TS_RE = re.compile(r"<\|\d{1,2}\.\d{2}\|>")
_SPECIAL_RE = re.compile(r"<\|[\w\.]{1,12}\|>")      # cool_dataset.py:35 (append handler)
_TOKEN_RE = re.compile(r"<\|[^|<>]+\|>")               # any <|...|> candidate for the tokenizer


# ------------------------------------------------------------------------------------------ files
def load_audio_fpaths(manifest_fpath: str, root: Optional[str] = None) -> List[str]:
    """cool_dataset.py:94-104: the manifest's first line is the root directory (ignored when `root`
    is given), every further line a path relative to it (whitespace-stripped)."""
    out = []
    with open(manifest_fpath, "r") as fr:
        first = fr.readline().strip()
        if root is None:
            root = first
        for line in fr:
            out.append(osp.join(root, line.strip()))
    return out


def decode_flac(data: bytes):
    """FLAC bytes -> (float64 samples [n] or [n, channels] scaled like soundfile.read, sample rate), via
    tw_flac_info / tw_flac_decode (frame CRCs checked; a malformed stream raises)."""
    import ctypes
    from ._native import call
    buf = np.frombuffer(data, dtype=np.uint8)
    info = np.zeros(4, dtype=np.int64)
    call("tw_flac_info", buf.ctypes.data, buf.size, info.ctypes.data)
    ch, sr, bps = int(info[0]), int(info[1]), int(info[2])
    frames = ctypes.c_int64(0)
    call("tw_flac_decode", buf.ctypes.data, buf.size, None, 0, ctypes.addressof(frames))
    out = np.empty(frames.value * ch, dtype=np.int32)
    call("tw_flac_decode", buf.ctypes.data, buf.size, out.ctypes.data, out.size, ctypes.addressof(frames))
    x = out.astype(np.float64) / float(1 << (bps - 1))
    return (x.reshape(-1, ch) if ch > 1 else x), sr


def read_audio(path: str):
    """-> (float64 samples in [-1, 1), sampling rate), like soundfile.read(path)."""
    try:
        import soundfile as sf  # the reference's reader (absent in this image)
        data, sr = sf.read(path)
        return np.asarray(data, dtype=np.float64), int(sr)
    except ImportError:
        pass
    ext = osp.splitext(path)[1].lower()
    if ext == ".flac":
        with open(path, "rb") as f:
            return decode_flac(f.read())
    if ext == ".npy":
        return np.load(path).astype(np.float64), SAMPLING_RATE
    if ext == ".wav":
        with wave.open(path, "rb") as w:
            n, ch, sw, sr = w.getnframes(), w.getnchannels(), w.getsampwidth(), w.getframerate()
            raw = w.readframes(n)
        if sw == 1:
            x = (np.frombuffer(raw, np.uint8).astype(np.float64) - 128.0) / 128.0
        elif sw == 2:
            x = np.frombuffer(raw, "<i2").astype(np.float64) / 32768.0
        elif sw == 3:
            b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = v.astype(np.float64) / float(1 << 23)
        elif sw == 4:
            x = np.frombuffer(raw, "<i4").astype(np.float64) / float(1 << 31)
        else:
            raise ValueError(f"{path}: unsupported sample width {sw}")
        if ch > 1:
            x = x.reshape(-1, ch)
        return x, sr
    raise RuntimeError(f"{path}: decoding {ext} needs the `soundfile` package (libsndfile), which is not "
                       f"installed here; WAV and .npy are read natively")


def read_transcript(txt_fpath: str) -> dict:
    """cool_dataset.py:63-83 (the .txt beside the audio file)."""
    with open(txt_fpath, "r") as fr:
        lines = fr.readlines()
    whisper_transcript = lines[0].strip().split("<|endoftext|>")[0]
    end_transcript = lines[2].strip()
    prev_transcript = lines[4].strip().split("<|endoftext|>")[0]
    f = {"whisper_transcript": whisper_transcript, "last_segment_transcript": end_transcript,
         "condition_on_prev": "<|startofprev|>" + prev_transcript}
    if "<|continued|>" in prev_transcript:
        ts = _TS_RE.findall(f["condition_on_prev"])
        if len(ts) > 1:
            last = ts[-1]
            f["condition_on_prev"] = f["condition_on_prev"].split(last)[0] + last
            # (the reference's following `.replace("<|continued|>", "")` discards its result: a no-op)
    return f


def trim_last_segment(feature: dict) -> dict:
    """cool_dataset.py:20-31: with more than one timestamp, keep the transcript up to its last
    timestamp and cut the audio at that time."""
    ts = _TS_RE.findall(feature["whisper_transcript"])
    if len(ts) > 1:
        last = ts[-1]
        feature["whisper_transcript"] = feature["whisper_transcript"].split(last)[0] + last
        cut = int(float(last[2:-2]) * SAMPLING_RATE)
        if cut < len(feature["audio"]["array"]):
            feature["audio"]["array"] = feature["audio"]["array"][:cut]
    return feature


def append_last_segment(feature: dict) -> dict:
    """cool_dataset.py:33-47 (see the module docstring: returns the feature)."""
    specials = _SPECIAL_RE.findall(feature["whisper_transcript"])
    if "<|continued|>" in specials:
        ts_before = specials[specials.index("<|continued|>") - 1]
        t = feature["whisper_transcript"].split(ts_before)[0]
        feature["whisper_transcript"] = t + feature["last_segment_transcript"] + "<|endoftext|>"
    else:
        t = feature["whisper_transcript"].split("<|endoftext|>")[0]
        feature["whisper_transcript"] = t + feature["last_segment_transcript"] + "<|endoftext|>"
    return feature


LAST_SEGMENT_HANDLERS = {"trim": trim_last_segment, "append": append_last_segment}


class CoolDataset:
    """Random-access view of a manifest (the reference streams it through
    IterableDataset.from_generator; items are identical)."""

    def __init__(self, manifest_fpath: str, root: Optional[str] = None, last_segment_handler: str = "trim",
                 audio_reader: Callable = read_audio):
        self.audio_fpaths = load_audio_fpaths(manifest_fpath, root)
        self.handler = LAST_SEGMENT_HANDLERS[last_segment_handler]
        self.audio_reader = audio_reader

    def __len__(self):
        return len(self.audio_fpaths)

    def __getitem__(self, i: int) -> dict:
        path = self.audio_fpaths[i]
        data, sr = self.audio_reader(path)
        f = read_transcript(osp.splitext(path)[0] + ".txt")
        f["audio"] = {"path": path, "sampling_rate": sr, "array": data}
        return self.handler(f)


# ------------------------------------------------------------------------------------ tokenizer
def whisper_special_tokens(n_languages: int = 99) -> dict:
    """Multilingual Whisper special-token ids (Appendix A of SURVEY.md; HF vocab order):
    <|endoftext|> 50257, <|startoftranscript|> 50258, language tokens from 50259 (<|en|>, <|zh|>, ...),
    <|translate|> 50358, <|transcribe|> 50359, <|startoflm|> 50360, <|startofprev|> 50361,
    <|nocaptions|> 50362, <|notimestamps|> 50363, <|0.00|> ... <|30.00|> 50364 ... 51864."""
    langs = ["en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca", "nl", "ar", "sv", "it", "id",
             "hi", "fi", "vi", "he", "uk", "el", "ms", "cs", "ro", "da", "hu", "ta", "no", "th", "ur", "hr", "bg",
             "lt", "la", "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn", "et", "mk", "br",
             "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw", "gl", "mr", "pa", "si", "km", "sn", "yo", "so",
             "af", "oc", "ka", "be", "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo", "ht", "ps", "tk", "nn", "mt",
             "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha", "ba", "jw", "su"][:n_languages]
    tab = {"<|endoftext|>": EOT, "<|startoftranscript|>": SOT}
    for i, l in enumerate(langs):
        tab[f"<|{l}|>"] = 50259 + i
    tab.update({"<|translate|>": 50358, "<|transcribe|>": TRANSCRIBE, "<|startoflm|>": 50360,
                "<|startofprev|>": STARTOFPREV, "<|nocaptions|>": 50362, "<|notimestamps|>": NOTIMESTAMPS})
    for i in range(1501):
        tab["<|%.2f|>" % (i * 0.02)] = NOTIMESTAMPS + 1 + i
    return tab


class WhisperTokenizerAdapter:
    """`tokenizer(text, add_special_tokens=...)` with WhisperTokenizerFast semantics for the parts the
    training path uses: Whisper special tokens (and the 1501 added timestamp tokens) are atomic; the
    text between them goes to `text_encoder` (the BPE: an HF tokenizer's encode without special
    tokens when its files exist, any str -> ids callable otherwise); add_special_tokens=True wraps
    the ids in the prefix tokens [SOT, <|lang|>, <|task|>] (+ <|notimestamps|> unless
    predict_timestamps) and <|endoftext|>.  Unknown <|...|> strings (e.g. <|continued|>) are text."""

    def __init__(self, text_encoder: Callable[[str], List[int]], language: Optional[str] = "zh",
                 task: Optional[str] = "transcribe", predict_timestamps: bool = True,
                 text_decoder: Optional[Callable[[List[int]], str]] = None):
        self.special = whisper_special_tokens()
        self.id_to_special = {v: k for k, v in self.special.items()}
        self.text_encoder, self.text_decoder = text_encoder, text_decoder
        self.set_prefix_tokens(language, task, predict_timestamps)
        self.pad_token_id = self.eos_token_id = EOT

    def set_prefix_tokens(self, language=None, task=None, predict_timestamps=None):
        if language is not None:
            self.language = language
        if task is not None:
            self.task = task
        if predict_timestamps is not None:
            self.predict_timestamps = predict_timestamps
        p = [SOT]
        if getattr(self, "language", None):
            p.append(self.special[f"<|{self.language}|>"])
        if getattr(self, "task", None):
            p.append(self.special[f"<|{self.task}|>"])
        if not self.predict_timestamps:
            p.append(NOTIMESTAMPS)
        self.prefix_tokens = p

    def timestamp_ids(self):
        return list(range(NOTIMESTAMPS + 1, NOTIMESTAMPS + 1 + 1501))

    def encode(self, text: str, add_special_tokens: bool = True) -> List[int]:
        ids: List[int] = []
        pos = 0
        for m in _TOKEN_RE.finditer(text):
            tok = m.group(0)
            if tok not in self.special:
                continue
            if m.start() > pos:
                ids.extend(self.text_encoder(text[pos:m.start()]))
            ids.append(self.special[tok])
            pos = m.end()
        if pos < len(text):
            ids.extend(self.text_encoder(text[pos:]))
        if add_special_tokens:
            ids = self.prefix_tokens + ids + [EOT]
        return ids

    def __call__(self, text, add_special_tokens: bool = True):
        class _Enc:
            pass
        e = _Enc()
        e.input_ids = self.encode(text, add_special_tokens)
        return e

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        out, run = [], []
        for t in (int(x) for x in ids):
            if t in self.id_to_special or t > NOTIMESTAMPS:
                if run:
                    out.append(self.text_decoder(run) if self.text_decoder else "")
                    run = []
                if not skip_special_tokens:
                    out.append(self.id_to_special.get(t, ""))
            elif t >= 0:
                run.append(t)
        if run:
            out.append(self.text_decoder(run) if self.text_decoder else "")
        return "".join(out)

    def batch_decode(self, batch, skip_special_tokens: bool = True, **kw) -> List[str]:
        return [self.decode(row, skip_special_tokens) for row in batch]


# ----------------------------------------------------------------------------------- sharding
def shard_micro_batches(n_items: int, batch_size: int, rank: int, world: int, order: Optional[Sequence[int]] = None,
                        with_real: bool = False):
    """Item indices of the micro-batches rank `rank` consumes: global micro-batch j holds stream
    positions [j*B, (j+1)*B); rank r takes j = k*world + r.  The last group of `world` micro-batches
    is completed from the start of the stream (accelerate even_batches), so all ranks get the same
    number of full micro-batches.  with_real=True also returns, per micro-batch, how many of its
    leading items are real (stream position < n_items) -- the rows accelerate's gather_for_metrics
    keeps on the last batch (it truncates the rank-major gathered rows to the dataset remainder)."""
    order = list(range(n_items)) if order is None else list(order)
    if not order:
        return ([], []) if with_real else []
    group = batch_size * world
    n_groups = -(-len(order) // group)
    need = n_groups * group
    stream = [order[i % len(order)] for i in range(need)]
    out, real = [], []
    for k in range(n_groups):
        j = k * world + rank
        out.append(stream[j * batch_size:(j + 1) * batch_size])
        real.append(max(0, min(batch_size, len(order) - j * batch_size)))
    return (out, real) if with_real else out


# -------------------------------------------------------------------------------- preparation
def prepare_train_batch(features: Sequence[dict], tokenizer, rng: np.random.Generator, *,
                        text_column: str = "whisper_transcript", timestamp_probability: float = 0.5,
                        condition_on_prev_probability: float = 0.2, max_label_length: int = 448,
                        is_multilingual: bool = True, collator: Optional[DataCollatorSpeechSeq2SeqWithPadding] = None):
    """Host side of prepare_train_dataset (:1207-1274) + collator for one micro-batch: token ids of
    the transcripts / prompts, label sampling (tw.data.prepare_labels), padding.  Returns
    (list of float32 waveforms, decoder_input_ids int64 [B, L-1], labels int64 [B, L-1])."""
    collator = collator or DataCollatorSpeechSeq2SeqWithPadding(max_target_length=max_label_length)
    tok_batch, prev_batch = [], []
    for f in features:
        s = f[text_column]
        tok_batch.append(tokenizer(s, add_special_tokens="<|transcribe|>" not in s).input_ids)
        p = f.get("condition_on_prev")
        prev_batch.append(tokenizer(p, add_special_tokens=False).input_ids if isinstance(p, str) else p)
    has_prev = any("condition_on_prev" in f for f in features)
    labels = prepare_labels(tok_batch, prev_batch, rng, timestamp_probability, condition_on_prev_probability,
                            max_label_length, is_multilingual, has_prev_column=has_prev)
    dec, lab = collator.collate_labels(labels)
    wavs = [np.asarray(f["audio"]["array"], dtype=np.float32) for f in features]
    return wavs, dec, lab


class DataFeed:
    """Per-rank prefetching feed: host preparation of the next `depth` micro-batches runs in a thread
    pool while the current step runs; `next()` copies the waveforms into pinned memory, ships them
    with one async H2D copy and runs tw_logmel on the GPU, returning the trainer's batch dict
    (conv_input bf16 [B, 3002, 80] for the conv stem, decoder_input_ids, labels on the device)."""

    def __init__(self, dataset, tokenizer, batch_size: int, *, rank: int = 0, world: int = 1, device=None,
                 seed: int = 42, epoch: int = 0, shuffle: bool = True, depth: int = 2, workers: int = 4,
                 skip_batches: int = 0, **prep_kw):
        from .feature_extraction import WhisperFeatureExtractor
        self.ds, self.tok, self.B = dataset, tokenizer, batch_size
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        order = list(range(len(dataset)))
        if shuffle:
            np.random.Generator(np.random.PCG64(seed + epoch)).shuffle(order)
        batches, real = shard_micro_batches(len(order), batch_size, rank, world, order, with_real=True)
        self.batches, self.n_real = batches[skip_batches:], real[skip_batches:]
        self.rng = np.random.Generator(np.random.PCG64([seed, epoch, rank]))
        self.prep_kw = prep_kw
        self.fe = WhisperFeatureExtractor(device=self.device)
        self.pool = cf.ThreadPoolExecutor(max_workers=workers)
        self.depth = depth
        self._futs: list = []
        self._next = 0

    def __len__(self):
        return len(self.batches)

    def _host(self, idx):
        feats = [self.ds[i] for i in idx]
        return feats

    def _submit(self):
        while len(self._futs) < self.depth and self._next < len(self.batches):
            self._futs.append((self.pool.submit(self._host, self.batches[self._next]), self.n_real[self._next]))
            self._next += 1

    def __iter__(self):
        return self

    def __next__(self):
        self._submit()
        if not self._futs:
            self.pool.shutdown(wait=False)
            raise StopIteration
        fut, n_real = self._futs.pop(0)
        feats = fut.result()
        self._submit()
        # label sampling stays on this thread: one rng, stream order (deterministic per rank)
        wavs, dec, lab = prepare_train_batch(feats, self.tok, self.rng, **self.prep_kw)
        n = 480000
        host = torch.zeros(len(wavs), n, dtype=torch.float32).pin_memory()
        for i, w in enumerate(wavs):
            m = min(len(w), n)
            host[i, :m] = torch.from_numpy(w[:m])
        wav = host.to(self.device, non_blocking=True)
        mel, conv = self.fe.extract(wav, want_conv_input=True)
        return {"conv_input": conv, "input_features": mel,
                "decoder_input_ids": dec.to(self.device, non_blocking=True),
                "labels": lab.to(self.device, non_blocking=True), "n_real": n_real}
