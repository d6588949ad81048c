"""Pseudo-labelling driver: the MI355X counterpart of `pseudo-labelling/initial_inference.py`
(BASELINE config 4).

Reference flow (initial_inference.py:56-119): read `audio_path` from a CSV manifest (`load_dataset`,
:33-36); per file, faster-whisper's BatchedInferencePipeline.transcribe(task="transcribe", language,
batch_size) (:38-52) cuts the audio into chunks (VAD speech regions merged up to `chunk_length`
seconds) and decodes the chunks in batches; one CSV per file (`<name>.csv`, header start,end,text;
times formatted "%.2f", :48-54, :58-64), written to `--output_dir`; a missing file is reported and
skipped, a failing one logged and skipped (:96-119).

Here: the same CLI flags and output files, on this engine — GPU log-mel (tw_logmel), the large-v2
encoder and the batched greedy KV-cache decoder (`model.generate`, HIP graph per step).  Chunks of
consecutive files share batches (a batch is filled across file boundaries), and with several ranks
each rank takes files rank, rank + N, ... (replicas, no collective).
Differences, by design or by what this image lacks (each stated where it applies):
  * no VAD: the silero model faster-whisper loads is not available offline and VAD is out of scope
     -> chunks are consecutive `chunk_length`-second windows of the file;
  * greedy decoding (BASELINE config 4 "batched greedy"; faster-whisper's own default is beam 5) with
    the HF prompt [SOT, <|lang|>, <|transcribe|>, <|notimestamps|>] and HF feature semantics (each
    chunk zero-padded to 30 s before the STFT), the arithmetic the decode tests pin to HF;
  * text: `tokenizers.Tokenizer.from_file(<model dir>/tokenizer.json)` decode of the ids below
    <|endoftext|> (faster-whisper Tokenizer.decode); without that file, --byte_level_text_tokenizer
    decodes ids < 256 as UTF-8 bytes (tests only).
"""
from __future__ import annotations

import argparse
import collections
import concurrent.futures as cf
import csv
import os
import sys
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

SR = 16000
EOT = 50257


def _bool(v):
    return str(v).lower() in ("1", "true", "yes", "y")


def parse_args(argv=None):
    """initial_inference.py:13-27 flags (same names and defaults where they apply)."""
    ap = argparse.ArgumentParser(description="Transcribe audio files with the tw engine (pseudo-labelling).")
    ap.add_argument("--dataset_path", type=str, default="/mnt/dataset_1T/tmp_dir/sample.tsv")
    ap.add_argument("--output_dir", type=str, default="/mnt/pseudo_label")
    ap.add_argument("--language", type=str, default="zh")
    ap.add_argument("--log_progress", type=_bool, default=True)
    ap.add_argument("--model_size_or_path", type=str, default="tiny",
                    help="HF-format model directory (config.json + model.safetensors)")
    ap.add_argument("--compute_type", type=str, default="default",
                    help="default / float16 -> the fp16 model (CTranslate2's CUDA default for a float16 checkpoint); "
                         "bfloat16 -> bf16; float32 -> the fp32 path")
    ap.add_argument("--chunk_length", type=int, default=5)
    ap.add_argument("--batch_size", type=int, default=64)
    ap.add_argument("--num_workers", type=int, default=8, help="host audio-decoding threads")
    ap.add_argument("--max_new_tokens", type=int, default=None)
    ap.add_argument("--byte_level_text_tokenizer", type=_bool, default=False)
    return ap.parse_args(argv)


def load_dataset(dataset_path: str) -> List[str]:
    """initial_inference.py:33-36: the `audio_path` column of the manifest (pandas.read_csv)."""
    import pandas as pd
    return pd.read_csv(dataset_path)["audio_path"].tolist()


def chunk_audio(wav: np.ndarray, sr: int, chunk_length: float) -> List[Tuple[float, float, np.ndarray]]:
    """Consecutive chunks of `chunk_length` seconds (the last one shorter) -> (start s, end s, samples)."""
    if sr != SR:
        raise ValueError(f"expected {SR} Hz audio, got {sr} Hz")
    wav = np.asarray(wav, dtype=np.float32)
    if wav.ndim > 1:                                     # channels averaged (faster-whisper decode_audio)
        wav = wav.mean(axis=1).astype(np.float32)
    step = int(round(chunk_length * sr))
    out = []
    for a in range(0, len(wav), step):
        b = min(len(wav), a + step)
        out.append((a / sr, b / sr, wav[a:b]))
    return out


def save_transcription_to_csv(rows: Sequence[dict], output_csv: str):
    """initial_inference.py:48-54."""
    with open(output_csv, "w", newline="", encoding="utf-8") as f:
        w = csv.DictWriter(f, fieldnames=["start", "end", "text"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


class ChunkTranscriber:
    """Batched greedy transcription of <= 30 s chunks: GPU log-mel of the zero-padded chunk, encoder,
    KV-cache greedy decode.  Returns the generated ids per chunk (eos and padding removed)."""

    def __init__(self, model, language: str = "zh", max_new_tokens: Optional[int] = None, device=None):
        from .feature_extraction import WhisperFeatureExtractor
        self.m = model
        self.fe = WhisperFeatureExtractor(device=device or model.device)
        self.language, self.max_new_tokens = language, max_new_tokens

    def __call__(self, chunks: Sequence[np.ndarray]) -> List[List[int]]:
        if not chunks:
            return []
        wav = self.fe.pad_waveforms(list(chunks))
        mel, _ = self.fe.extract(wav, want_conv_input=False)
        ids = self.m.generate(mel, language=self.language, task="transcribe", max_new_tokens=self.max_new_tokens)
        out = []
        for row in ids.tolist():
            k = row.index(EOT) if EOT in row else len(row)
            out.append(row[:k])
        return out


def transcribe_files(paths: Sequence[str], transcribe: Callable[[Sequence[np.ndarray]], List[List[int]]],
                     decode: Callable[[List[int]], str], chunk_length: float, batch_size: int,
                     read_audio: Callable[[str], Tuple[np.ndarray, int]], num_workers: int = 8,
                     log: Callable[[str], None] = print,
                     on_done: Optional[Callable[[str, List[dict]], None]] = None,
                     max_ahead: Optional[int] = None) -> Dict[str, Optional[List[dict]]]:
    """-> {path: rows or None (missing / failed file)}.  Files are decoded on `num_workers` host threads
    ahead of the GPU, at most `max_ahead` (default 2 x num_workers) files in flight, so host memory holds a
    bounded number of decoded waveforms whatever the manifest size; chunks of consecutive files fill
    batches of `batch_size` across file boundaries.  `on_done(path, rows)` runs as soon as a file's last
    chunk is transcribed (the reference writes each CSV when its file finishes, initial_inference.py:106-
    115).  A batch whose transcription or text decoding raises is retried one file at a time; a file whose own
    chunks raise is failed (logged, result None, its other chunks dropped) and the run goes on (:116-119)."""
    results: Dict[str, Optional[List[dict]]] = {}
    pending: List[Tuple[str, float, float, np.ndarray]] = []
    counts: Dict[str, int] = {}
    rows: Dict[str, List[dict]] = {}

    def finish(p, r):
        results[p] = r
        if on_done is not None and r is not None:
            on_done(p, r)

    def fail(bad, e):
        for p in bad:
            log(f"Failed to transcribe {p}, error: {e}")
            rows.pop(p, None)
            counts.pop(p, None)
            results[p] = None
        pending[:] = [c for c in pending if c[0] not in set(bad)]

    def run(batch):
        toks = transcribe([c[3] for c in batch])
        return [decode(t) for t in toks]

    def flush(force=False):
        while pending and (force or len(pending) >= batch_size):
            batch = pending[:batch_size]
            del pending[:batch_size]
            files = list(dict.fromkeys(c[0] for c in batch))
            try:
                done = list(zip(batch, run(batch)))
            except Exception as e:              # noqa: BLE001 -- log the failing files and go on
                if len(files) == 1:
                    fail(files, e)
                    continue
                # chunks of several files share the batch: retry it one file at a time, so only a file whose own
                # chunks raise is failed (the reference fails only the file that raised, :106-119)
                done = []
                for p in files:
                    sub = [c for c in batch if c[0] == p]
                    try:
                        done.extend(zip(sub, run(sub)))
                    except Exception as e1:     # noqa: BLE001
                        fail([p], e1)
            for (p, s, e, _), t in done:
                if p not in rows:               # failed in an earlier batch
                    continue
                rows[p].append({"start": f"{s:.2f}", "end": f"{e:.2f}", "text": t})
                if len(rows[p]) == counts[p]:
                    counts.pop(p)
                    finish(p, rows.pop(p))

    def load(p):
        if not os.path.exists(p):
            return p, None, "missing"
        try:
            wav, sr = read_audio(p)
            return p, chunk_audio(wav, sr, chunk_length), None
        except Exception as e:                  # noqa: BLE001 -- the reference logs and skips the file
            return p, None, str(e)

    ahead = max(1, max_ahead if max_ahead is not None else 2 * max(1, num_workers))
    with cf.ThreadPoolExecutor(max(1, num_workers)) as ex:
        futs: "collections.deque[cf.Future]" = collections.deque()
        it = iter(paths)

        def refill():
            while len(futs) < ahead:
                try:
                    futs.append(ex.submit(load, next(it)))
                except StopIteration:
                    return

        refill()
        while futs:
            p, chunks, err = futs.popleft().result()
            refill()                            # keep the read-ahead window full while the GPU works
            log(f"Processing: {p}")
            if err == "missing":
                log(f"File not found: {p}")
                results[p] = None
                continue
            if err is not None:
                log(f"Failed to transcribe {p}, error: {err}")
                results[p] = None
                continue
            if not chunks:
                finish(p, [])
                continue
            counts[p], rows[p] = len(chunks), []
            pending.extend((p, s, e, w) for s, e, w in chunks)
            del chunks
            flush()
        flush(force=True)
    return results


def load_text_decoder(args) -> Callable[[List[int]], str]:
    if args.byte_level_text_tokenizer:
        return lambda ids: bytes(i for i in ids if i < 256).decode("utf-8", "ignore")
    path = os.path.join(args.model_size_or_path, "tokenizer.json")
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not found (faster-whisper reads the checkpoint's tokenizer.json); pass "
                                "--byte_level_text_tokenizer True to decode byte ids (tests)")
    import tokenizers
    tok = tokenizers.Tokenizer.from_file(path)
    return lambda ids: tok.decode([i for i in ids if i < EOT])


def main(argv=None):
    args = parse_args(argv)
    print(args)
    from .dataset import read_audio
    from .modeling import WhisperForConditionalGeneration
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    ct = args.compute_type
    compute = "fp32" if ct in ("float32", "fp32") else "bf16" if ct in ("bfloat16", "bf16") else "fp16"
    dtype = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[compute]
    model = WhisperForConditionalGeneration.from_pretrained(
        args.model_size_or_path, torch_dtype=dtype, device=torch.device("cuda", local), compute=compute)
    print(f"Using device: cuda:{local} ({compute})", flush=True)
    decode = load_text_decoder(args)
    tr = ChunkTranscriber(model, args.language, args.max_new_tokens)
    paths = load_dataset(args.dataset_path)[rank::world]
    os.makedirs(args.output_dir, exist_ok=True)
    def write(p, r):
        out = os.path.join(args.output_dir, os.path.splitext(os.path.basename(p))[0] + ".csv")
        save_transcription_to_csv(r, out)
        print(f"Transcription completed: {out}", flush=True)

    res = transcribe_files(paths, tr, decode, args.chunk_length, args.batch_size, read_audio, args.num_workers,
                           log=(lambda s: print(s, flush=True)) if args.log_progress else (lambda s: None),
                           on_done=write)
    return res


if __name__ == "__main__":
    sys.exit(0 if main() is not None else 1)
