"""Host side of the §8f rows 1-2 (CPU): NTU-COOL manifest / transcript parsing with the last-segment
trim, native WAV decoding, the special-token tokenizer adapter, per-rank micro-batch sharding,
training-batch preparation against the oracle's label restatement, and the MER metric.

Parity notes: the reference's dataset module (dataset/cool_dataset.py) imports soundfile at module
load and utils/evaluation.py imports opencc / editdistance / pypinyin, none of which is installed, so
both are restated from source text and pinned here on hand-worked cases (file:line in tw.dataset /
tw.evaluation docstrings)."""
import os
import random
import wave

import numpy as np
import pytest
import torch

from oracle import labels as L
from tw import dataset as D
from tw import evaluation as E


def _write_clip(dirpath, name, samples, transcript, last_seg="", prev="", sr=16000):
    wav = os.path.join(dirpath, name + ".wav")
    with wave.open(wav, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes((np.clip(samples, -1, 0.99997) * 32768).astype("<i2").tobytes())
    with open(os.path.join(dirpath, name + ".txt"), "w") as f:
        f.write(transcript + "\n\n" + last_seg + "\n\n" + prev + "\n")
    return wav


def test_manifest_and_transcript(tmp_path):
    root = tmp_path / "corpus"
    root.mkdir()
    x = 0.25 * np.sin(np.arange(16000 * 3) / 16000 * 2 * np.pi * 440)
    _write_clip(str(root), "a", x, "<|0.00|>hello<|1.00|><|1.00|>world<|2.50|><|2.50|><|continued|><|endoftext|>",
                "<|0.00|>tail<|1.20|>", "<|0.00|>before<|3.00|><|3.00|>more<|4.00|><|continued|><|endoftext|>")
    _write_clip(str(root), "b", x[:8000], "<|startoftranscript|><|zh|><|transcribe|>你好<|endoftext|>")
    man = tmp_path / "m.tsv"
    man.write_text(f"{root}\na.wav\nb.wav\n")
    assert D.load_audio_fpaths(str(man)) == [str(root / "a.wav"), str(root / "b.wav")]
    assert D.load_audio_fpaths(str(man), root="/x") == ["/x/a.wav", "/x/b.wav"]
    ds = D.CoolDataset(str(man))
    a = ds[0]
    # trim handler: transcript cut after the LAST timestamp, audio cut at 2.50 s
    assert a["whisper_transcript"] == "<|0.00|>hello<|1.00|><|1.00|>world<|2.50|>"
    assert len(a["audio"]["array"]) == int(2.5 * 16000)
    assert a["last_segment_transcript"] == "<|0.00|>tail<|1.20|>"
    # previous transcript: <|continued|> present, >1 timestamps -> cut after the last one
    assert a["condition_on_prev"] == "<|startofprev|><|0.00|>before<|3.00|><|3.00|>more<|4.00|>"
    b = ds[1]
    assert b["whisper_transcript"] == "<|startoftranscript|><|zh|><|transcribe|>你好"
    assert len(b["audio"]["array"]) == 8000                   # 0 or 1 timestamps: untouched
    np.testing.assert_allclose(b["audio"]["array"], np.round(x[:8000] * 32768) / 32768, atol=1 / 32768)
    # append handler (restated with a return)
    f = {"whisper_transcript": "<|0.00|>a<|9.00|><|continued|>", "last_segment_transcript": "<|9.00|>b<|11.00|>"}
    assert D.append_last_segment(dict(f))["whisper_transcript"] == "<|0.00|>a<|9.00|>b<|11.00|><|endoftext|>"


def test_tokenizer_adapter():
    tok = D.WhisperTokenizerAdapter(lambda s: list(s.encode("utf-8")), language="zh", task="transcribe",
                                    predict_timestamps=True)
    assert tok.prefix_tokens == [50258, 50260, 50359]
    ids = tok("<|0.00|>hi<|1.02|>", add_special_tokens=True).input_ids
    assert ids == [50258, 50260, 50359, 50364, 104, 105, 50364 + 51, 50257]
    # already carrying the task token (the reference passes add_special_tokens=False then)
    s = "<|startoftranscript|><|zh|><|transcribe|>ok<|continued|>"
    ids = tok(s, add_special_tokens="<|transcribe|>" not in s).input_ids
    assert ids[:3] == [50258, 50260, 50359]
    assert ids[3:] == list(b"ok<|continued|>")                 # unknown <|...|> is text
    tok.set_prefix_tokens(predict_timestamps=False)
    assert tok.prefix_tokens == [50258, 50260, 50359, 50363]
    assert tok.timestamp_ids()[0] == 50364 and tok.timestamp_ids()[-1] == 51864
    assert D.whisper_special_tokens()["<|30.00|>"] == 51864


def test_shard_micro_batches():
    # rank r of N takes global micro-batch k*N + r; last group completed from the stream start
    B, N = 2, 3
    shards = [D.shard_micro_batches(13, B, r, N) for r in range(N)]
    assert all(len(s) == 3 for s in shards)                    # ceil(13 / 6) groups
    stream = [i % 13 for i in range(18)]
    for r in range(N):
        for k, mb in enumerate(shards[r]):
            j = k * N + r
            assert mb == stream[j * B:(j + 1) * B]
    seen = sorted(i for s in shards for mb in s for i in mb)
    assert set(seen) == set(range(13))
    assert D.shard_micro_batches(0, 4, 0, 2) == []
    # real-item counts: stream positions < 13 are real, the wrapped tail is duplicates
    for r in range(N):
        mbs, real = D.shard_micro_batches(13, B, r, N, with_real=True)
        assert mbs == shards[r]
        for k, n in enumerate(real):
            j = k * N + r
            assert n == sum(1 for pos in range(j * B, (j + 1) * B) if pos < 13)
    total_real = sum(n for r in range(N) for n in D.shard_micro_batches(13, B, r, N, with_real=True)[1])
    assert total_real == 13


def test_prepare_train_batch_matches_oracle():
    tok = D.WhisperTokenizerAdapter(lambda s: list(s.encode("utf-8")), language="zh", task="transcribe")
    feats = []
    for i in range(4):
        txt = "<|startoftranscript|><|zh|><|transcribe|><|0.00|>" + "x" * (10 + 7 * i) + "<|2.00|>"
        feats.append({"whisper_transcript": txt, "condition_on_prev": "<|startofprev|>prev text %d" % i,
                      "audio": {"array": np.zeros(1000 + i)}})
    wavs, dec, lab = D.prepare_train_batch(feats, tok, np.random.Generator(np.random.PCG64(3)),
                                           timestamp_probability=0.5, condition_on_prev_probability=0.5)
    # the same label sampling through the oracle restatement (same rng stream)
    toks = [tok(f["whisper_transcript"], add_special_tokens=False).input_ids for f in feats]
    prevs = [tok(f["condition_on_prev"], add_special_tokens=False).input_ids for f in feats]
    ref = L.prepare_labels(toks, prevs, np.random.Generator(np.random.PCG64(3)), 0.5, 0.5, 448, True,
                           has_prev_column=True)
    rd, rl = L.collate(ref)
    assert torch.equal(dec, torch.from_numpy(rd)) and torch.equal(lab, torch.from_numpy(rl))
    assert dec.shape == (4, 447) and [len(w) for w in wavs] == [1000, 1001, 1002, 1003]


def test_levenshtein_exact():
    rnd = random.Random(0)

    def naive(a, b):
        d = list(range(len(b) + 1))
        for i in range(1, len(a) + 1):
            prev, d[0] = d[0], i
            for j in range(1, len(b) + 1):
                cur = min(d[j] + 1, d[j - 1] + 1, prev + (a[i - 1] != b[j - 1]))
                prev, d[j] = d[j], cur
        return d[-1]
    for _ in range(200):
        a = [rnd.choice("abcd") for _ in range(rnd.randint(0, 30))]
        b = [rnd.choice("abcd") for _ in range(rnd.randint(0, 30))]
        assert E.levenshtein(a, b) == naive(a, b)
        s, d, i, n = E.cal_single_complete_mer(a, b)
        assert s + d + i == naive(a, b) and n == len(a)


def test_mix_error_rate():
    m = E.MixErrorRate(converter=None)
    # CJK characters are units, English words are units, punctuation and spaces separate
    assert m._from_str_to_list("我們用 Python，寫code!") == ["我", "們", "用", "Python", "寫", "code"]
    assert m._from_str_to_list("a[b]c") == ["abc"]               # '[' ']' are not separators (reference quirk)
    assert m.compute(["我們用 Python"], ["我們用 python"]) == pytest.approx(1 / 4)
    assert m.compute(["", ""], ["", ""]) == 1.0                  # no reference -> empty_error_rate
    m2 = E.MixErrorRate(converter=None, separate_language=True, count_repetitive_hallucination=True)
    r = m2.compute(["今天 is good day"], ["今天天 is a good day"])
    assert r["MER"] == pytest.approx(2 / 7) and r["EN WER"] == pytest.approx(1 / 4)
    assert r["ZH CER"] == pytest.approx(1 / 3)
    assert E.MixErrorRate._count_repetitive_hallucination("abcdef" * 6) == 1
    conv = E.MixErrorRate(converter=lambda c: {"們": "们"}.get(c, c))
    assert conv.compute(["我們"], ["我们"]) == 0.0


def test_compute_metrics_with_adapter():
    tok = D.WhisperTokenizerAdapter(lambda s: list(s.encode("utf-8")), language="zh", task="transcribe",
                                    text_decoder=lambda ids: bytes(ids).decode("utf-8", "ignore"))
    lab = tok("hello world", add_special_tokens=True).input_ids
    pred = tok("hello word", add_special_tokens=True).input_ids
    labels = [lab[1:] + [-100, -100]]
    wer, pred_str, label_str, npred, nlab = E.compute_metrics([pred[1:]], labels, tok, E.MixErrorRate(converter=None))
    assert label_str == ["hello world"] and pred_str == ["hello word"]
    assert wer["wer_ortho"] == pytest.approx(50.0) and wer["wer"] == pytest.approx(50.0)


def test_cli_parser_accepts_reference_flags():
    from tw.run_distillation import build_parser
    a = build_parser().parse_args([
        "--model_name_or_path", "s", "--teacher_model_name_or_path", "t", "--output_dir", "o",
        "--train_dataset_manifest", "m.tsv", "--per_device_train_batch_size", "32", "--gradient_accumulation_steps",
        "2", "--learning_rate", "1e-4", "--lr_scheduler_type", "constant_with_warmup", "--warmup_steps", "50",
        "--max_steps", "120000", "--timestamp_probability", "0.5", "--condition_on_prev_probability", "0.2",
        "--freeze_encoder", "True", "--freeze_embed_positions", "True", "--mix_lang_emb", "True", "--dtype",
        "bfloat16", "--wandb_project", "x", "--is_prefiltered", "True", "--streaming", "True"])
    assert a.freeze_encoder and a.mix_lang_emb and a.per_device_train_batch_size == 32 and a.max_steps == 120000
