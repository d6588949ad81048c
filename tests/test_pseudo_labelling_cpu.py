"""Pseudo-labelling driver host logic (tw/pseudo_labelling.py vs pseudo-labelling/initial_inference.py):
manifest reading, chunking, batches filled across file boundaries, missing / failing / empty files,
CSV layout.  The transcriber is a stand-in here (the GPU path: tests/test_pseudo_labelling_gpu.py)."""
import csv
import os
import sys
import wave

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "taiwan-whisper_amd"))

from tw import pseudo_labelling as pl  # noqa: E402


def _wav(path, x, sr=16000):
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes((np.clip(x, -1, 1 - 2 ** -15) * 32768).astype("<i2").tobytes())


def test_chunk_audio():
    x = np.arange(16000 * 12, dtype=np.float32) / 1e6
    ch = pl.chunk_audio(x, 16000, 5)
    assert [(s, e) for s, e, _ in ch] == [(0.0, 5.0), (5.0, 10.0), (10.0, 12.0)]
    assert np.array_equal(np.concatenate([c for _, _, c in ch]), x)
    st = np.stack([x, -x], 1)
    assert np.allclose(pl.chunk_audio(st, 16000, 5)[0][2], 0)
    with pytest.raises(ValueError):
        pl.chunk_audio(x, 8000, 5)
    assert pl.chunk_audio(np.zeros(0, np.float32), 16000, 5) == []


def test_transcribe_files_batches_across_files(tmp_path):
    from tw.dataset import read_audio
    lens = {"a": 12.0, "b": 3.0, "c": 0.0, "d": 11.0}
    paths = []
    for k, secs in lens.items():
        p = tmp_path / f"{k}.wav"
        n = int(secs * 16000)
        _wav(p, np.full(n, 0.25 * (ord(k) - 96) / 4, dtype=np.float32))
        paths.append(str(p))
    paths.insert(2, str(tmp_path / "missing.wav"))
    bad = tmp_path / "bad.wav"
    bad.write_bytes(b"not a wav")
    paths.append(str(bad))
    calls = []

    def fake(chunks):
        calls.append(len(chunks))
        # "tokens" = the chunk's length in samples and its first value (identifies the chunk)
        return [[len(c), int(round(float(c[0]) * 1000))] for c in chunks]
    res = pl.transcribe_files(paths, fake, lambda ids: " ".join(map(str, ids)), 5, 4, read_audio, num_workers=3,
                              log=lambda s: None)
    assert calls == [4, 3]                         # a: 3 chunks, b: 1, d: 3 -> 7 chunks: batches of 4 + 3
    assert res[str(tmp_path / "missing.wav")] is None and res[str(bad)] is None
    assert res[str(tmp_path / "c.wav")] == []
    a = res[str(tmp_path / "a.wav")]
    assert [(r["start"], r["end"]) for r in a] == [("0.00", "5.00"), ("5.00", "10.00"), ("10.00", "12.00")]
    assert a[0]["text"] == "80000 62" and a[2]["text"] == "32000 62"
    assert res[str(tmp_path / "b.wav")] == [{"start": "0.00", "end": "3.00", "text": "48000 125"}]
    d = res[str(tmp_path / "d.wav")]
    assert [r["end"] for r in d] == ["5.00", "10.00", "11.00"] and d[-1]["text"] == "16000 250"
    out = tmp_path / "a.csv"
    pl.save_transcription_to_csv(a, str(out))
    with open(out, newline="", encoding="utf-8") as f:
        rows = list(csv.reader(f))
    assert rows[0] == ["start", "end", "text"] and rows[1] == ["0.00", "5.00", "80000 62"]


def test_load_dataset(tmp_path):
    m = tmp_path / "m.csv"
    m.write_text("audio_path,duration\n/x/1.flac,3\n/x/2.flac,4\n")
    assert pl.load_dataset(str(m)) == ["/x/1.flac", "/x/2.flac"]


def test_transcribe_files_bounded_readahead_and_failures(tmp_path):
    """the read-ahead is bounded (2 x workers files in flight), each file is reported as soon as
    its last chunk is done (the reference writes each CSV when its file finishes), and a batch whose
    transcription raises is retried one file at a time, so only the file that raised fails
    (initial_inference.py:116-119)."""
    import threading
    import time
    n_files = 40
    paths = [f"/virtual/{i}.wav" for i in range(n_files)]
    lock = threading.Lock()
    state = {"live": 0, "peak": 0, "consumed": 0}

    def read_audio(p):
        with lock:
            state["live"] += 1
            state["peak"] = max(state["peak"], state["live"] - state["consumed"])
        time.sleep(0.002)
        i = int(os.path.basename(p).split(".")[0])
        return np.full(16000 * (1 + i % 3), i / 100.0, dtype=np.float32), 16000

    done_order = []

    def fake(chunks):
        state["consumed"] += len({round(float(c[0]) * 100) for c in chunks})
        ids = [int(round(float(c[0]) * 100)) for c in chunks]
        if 7 in ids:
            raise RuntimeError("synthetic GPU error")
        return [[i] for i in ids]
    real_exists = os.path.exists
    try:
        pl.os.path.exists = lambda p: p.startswith("/virtual/") or real_exists(p)
        res = pl.transcribe_files(paths, fake, lambda t: str(t[0]), 1, 3, read_audio, num_workers=2,
                                  log=lambda s: None, on_done=lambda p, r: done_order.append(p))
    finally:
        pl.os.path.exists = real_exists
    # only file 7 failed (its batch neighbours completed on the per-file retry); everything else once, in order
    failed = [p for p in paths if res[p] is None]
    assert failed == [paths[7]]
    assert done_order == [p for p in paths if res[p] is not None]
    for i, p in enumerate(paths):
        if res[p] is not None:
            assert len(res[p]) == 1 + i % 3 and all(r["text"] == str(i) for r in res[p])
    # read-ahead bound: loads started but not yet consumed never exceed the window (+ the batch in hand)
    assert state["peak"] <= 2 * 2 + 3
