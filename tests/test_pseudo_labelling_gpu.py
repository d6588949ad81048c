"""Pseudo-labelling entry point on the GPU (tw/pseudo_labelling.main, initial_inference.py flags):
a micro-config checkpoint directory, a CSV manifest of three WAV files (one missing), chunk_length 5,
batch_size 3 (batches span files).  Every CSV row must equal the transcription of the same chunk in the
same batch composition by ChunkTranscriber directly (the batched greedy path, deterministic kernels),
with the reference's start/end formatting; the missing file is skipped."""
import csv
import os
import wave

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _wav(path, x):
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes((np.clip(x, -1, 1 - 2 ** -15) * 32768).astype("<i2").tobytes())


def test_pseudo_labelling_entry_point(tmp_path):
    from oracle import logmel
    from oracle.weights import CONFIGS, make_weights
    from tw import pseudo_labelling as pl
    from tw.config import GenerationConfig, WhisperConfig
    from tw.dataset import read_audio
    from tw.modeling import WhisperForConditionalGeneration
    cfg = CONFIGS["micro"]
    m = WhisperForConditionalGeneration.from_state_dict(
        WhisperConfig(**cfg), {k: torch.from_numpy(v) for k, v in make_weights(cfg, 2).items()}, dtype=torch.bfloat16)
    m.generation_config = GenerationConfig(suppress_tokens=[], begin_suppress_tokens=[220, 50257])
    ck = tmp_path / "ckpt"
    m.save_pretrained(str(ck))
    with open(ck / "generation_config.json", "w") as f:
        import json
        json.dump(dict(m.generation_config), f)
    files = []
    for i, secs in enumerate((12.0, 4.0, 9.5)):
        p = tmp_path / f"clip{i}.wav"
        _wav(p, logmel.synthetic_clip(10 + i, secs))
        files.append(str(p))
    files.insert(1, str(tmp_path / "missing.wav"))
    man = tmp_path / "manifest.csv"
    man.write_text("audio_path\n" + "\n".join(files) + "\n")
    out = tmp_path / "out"
    res = pl.main(["--dataset_path", str(man), "--output_dir", str(out), "--model_size_or_path", str(ck),
                   "--chunk_length", "5", "--batch_size", "3", "--num_workers", "2", "--max_new_tokens", "24",
                   "--byte_level_text_tokenizer", "True", "--log_progress", "False"])
    assert res[files[1]] is None and not (out / "missing.csv").exists()
    assert sorted(os.listdir(out)) == ["clip0.csv", "clip1.csv", "clip2.csv"]
    # the same chunks, the same batches, through ChunkTranscriber directly
    chunks = []
    for p in (files[0], files[2], files[3]):
        w, sr = read_audio(p)
        chunks += [(p, s, e, c) for s, e, c in pl.chunk_audio(w, sr, 5)]
    assert len(chunks) == 3 + 1 + 2
    # --compute_type default -> the fp16 model (CTranslate2's CUDA default for a float16 checkpoint)
    m2 = WhisperForConditionalGeneration.from_pretrained(str(ck), torch_dtype=torch.float16)
    assert m2.compute == "fp16"
    tr = pl.ChunkTranscriber(m2, "zh", 24)
    dec = pl.load_text_decoder(pl.parse_args(["--byte_level_text_tokenizer", "True"]))
    want = {}
    for i in range(0, len(chunks), 3):
        batch = chunks[i:i + 3]
        for (p, s, e, _), ids in zip(batch, tr([c[3] for c in batch])):
            assert 0 < len(ids) <= 24
            want.setdefault(p, []).append([f"{s:.2f}", f"{e:.2f}", dec(ids)])
    for p in (files[0], files[2], files[3]):
        with open(out / (os.path.splitext(os.path.basename(p))[0] + ".csv"), newline="", encoding="utf-8") as f:
            rows = list(csv.reader(f))
        assert rows[0] == ["start", "end", "text"]
        assert rows[1:] == want[p], p
    assert [r[1] for r in want[files[3]]] == ["5.00", "9.50"]
