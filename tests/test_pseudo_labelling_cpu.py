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
