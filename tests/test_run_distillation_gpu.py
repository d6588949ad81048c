"""End to end through the reference-style entry point (tw/run_distillation.py) on the GPU: a micro
teacher/student pair saved as HF directories, an NTU-COOL style manifest of WAV clips with 5-line
transcripts, the prefetching per-rank feed with GPU log-mel, train steps, accelerate-layout
checkpoints with rotation, eval (eval_step metrics + greedy generate + MER) and a resume that
continues from the last checkpoint.  Also checks the feed against the oracle's host path: the GPU
log-mel of the fed batch equals the oracle log-mel of the same trimmed waveforms."""
import json
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


def _corpus(root, n=6, sr=16000):
    os.makedirs(root, exist_ok=True)
    names = []
    for i in range(n):
        secs = 2.0 + 0.5 * i
        t = np.arange(int(secs * sr)) / sr
        x = 0.3 * np.sin(2 * np.pi * (200 + 40 * i) * t)
        with wave.open(os.path.join(root, f"c{i}.wav"), "wb") as w:
            w.setnchannels(1)
            w.setsampwidth(2)
            w.setframerate(sr)
            w.writeframes((x * 32767).astype("<i2").tobytes())
        body = "<|0.00|>" + "ab" * (3 + i) + "<|1.00|><|1.00|>" + "cd" * (2 + i) + "<|1.80|>"
        with open(os.path.join(root, f"c{i}.txt"), "w") as f:
            f.write("<|startoftranscript|><|zh|><|transcribe|>" + body + "<|endoftext|>\n\n<|0.00|>x<|0.50|>\n\n"
                    + "<|0.00|>prev" + str(i) + "<|1.00|><|endoftext|>\n")
        names.append(f"c{i}.wav")
    man = os.path.join(root, "manifest.tsv")
    with open(man, "w") as f:
        f.write(root + "\n" + "\n".join(names) + "\n")
    return man


def _model_dirs(tmp):
    from oracle.weights import CONFIGS, make_weights
    from tw.config import WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    cfg = CONFIGS["micro"]
    tc = WhisperConfig(**cfg)
    out = []
    for seed, name in ((2, "teacher"), (1, "student")):
        w = make_weights(cfg, seed)
        m = WhisperForConditionalGeneration.from_state_dict(tc, {k: torch.from_numpy(v) for k, v in w.items()},
                                                            dtype=torch.float32)
        d = os.path.join(tmp, name)
        m.save_pretrained(d)
        out.append(d)
    return out


def test_feed_batches_match_host_path(tmp_path):
    from oracle import logmel
    from tw import dataset as D
    man = _corpus(str(tmp_path / "corpus"))
    ds = D.CoolDataset(man)
    tok = D.WhisperTokenizerAdapter(lambda s: list(s.encode("utf-8")), language="zh")
    feed = D.DataFeed(ds, tok, 2, rank=1, world=2, device="cuda", seed=7, shuffle=False, workers=2,
                      timestamp_probability=1.0, condition_on_prev_probability=0.0)
    assert len(feed) == 2                                      # 6 clips, B=2, N=2 -> 2 groups
    batch = next(feed)
    idx = feed.batches[0]
    assert idx == [2, 3]                                       # rank 1 takes global micro-batch 1
    wavs = [ds[i]["audio"]["array"].astype(np.float32) for i in idx]
    ref = torch.from_numpy(logmel.log_mel_batch(wavs))
    assert float((batch["input_features"].cpu() - ref).abs().max()) < 2e-4
    assert batch["conv_input"].shape == (2, 3002, 80) and batch["labels"].shape == (2, 447)
    # labels: no prompt (p=0), timestamps kept (p=1): the transcript's ids, shifted, -100 padded
    ids = tok(ds[2]["whisper_transcript"], add_special_tokens=False).input_ids
    lab = batch["labels"][0].cpu()
    n = len(ids) - 1
    assert lab[:n].tolist() == ids[1:] and bool((lab[n:] == -100).all())


def test_entry_point_train_eval_resume(tmp_path):
    from tw.run_distillation import main
    teacher, student = _model_dirs(str(tmp_path))
    man = _corpus(str(tmp_path / "corpus"))
    out = str(tmp_path / "out")
    common = ["--model_name_or_path", student, "--teacher_model_name_or_path", teacher, "--output_dir", out,
              "--train_dataset_manifest", man, "--eval_dataset_manifest", man, "--per_device_train_batch_size", "2",
              "--per_device_eval_batch_size", "3", "--learning_rate", "1e-4", "--lr_scheduler_type",
              "constant_with_warmup", "--warmup_steps", "1", "--save_steps", "2", "--save_total_limit", "1",
              "--logging_steps", "1", "--freeze_encoder", "True", "--dtype", "bfloat16", "--language", "zh",
              "--timestamp_probability", "0.5", "--condition_on_prev_probability", "0.2", "--do_eval", "True",
              "--predict_with_generate", "True", "--max_label_length", "64", "--byte_level_text_tokenizer", "True",
              "--dataloader_num_workers", "2", "--streaming", "False"]
    res = main(common + ["--max_steps", "3", "--eval_steps", "3"])
    hist = res["train"]
    assert [h["step"] for h in hist] == [1, 2, 3]
    ev = res["eval"]
    assert len(ev) == 1 and ev[0]["step"] == 3 and np.isfinite(ev[0]["loss"]) and 0 <= ev[0]["wer"]
    assert all(np.isfinite(h["loss"]) and h["loss"] > 0 for h in hist)
    ck = sorted(d for d in os.listdir(out) if d.startswith("checkpoint-"))
    assert ck == ["checkpoint-3-epoch-0"]                      # save_total_limit 1 rotated checkpoint-2 away
    assert os.path.exists(os.path.join(out, ck[0], "optimizer.bin"))
    assert os.path.exists(os.path.join(out, "model.safetensors"))
    # best-checkpoint only when wer < 100 (the reference starts from best_wer = 100.0 and compares with <)
    assert os.path.exists(os.path.join(out, "best-checkpoint-epoch-0", "best_steps.txt")) == (ev[0]["wer"] < 100.0)
    # resume: continues at step 4 from checkpoint-3 (one epoch = 3 steps, so a new epoch)
    hist2 = main(common + ["--max_steps", "4", "--eval_steps", "100"])["train"]
    assert [h["step"] for h in hist2] == [4]
    from oracle.weights import CONFIGS
    with open(os.path.join(out, "config.json")) as f:
        assert json.load(f)["d_model"] == CONFIGS["micro"]["d_model"]


def test_partial_accumulation_steps_at_end_of_dataloader():
    """accelerate syncs at end_of_dataloader: with accum 2 and 3 micro-batches in an epoch the third
    micro-batch's (1/accum-scaled) gradient is applied by a second update instead of leaking into the
    next epoch's accumulation."""
    from oracle import labels as L
    from oracle.weights import CONFIGS, make_weights
    from tw.config import WhisperConfig
    from tw.distill import DistillationTrainer
    from tw.modeling import WhisperForConditionalGeneration
    cfg = CONFIGS["micro"]
    tc = WhisperConfig(**cfg)
    dev = torch.device("cuda", 0)
    mk = lambda seed, dt: WhisperForConditionalGeneration.from_state_dict(
        tc, {k: torch.from_numpy(v) for k, v in make_weights(cfg, seed).items()}, dtype=dt, device=dev)
    s, t = mk(1, torch.float32), mk(2, torch.bfloat16)
    tr = DistillationTrainer(s, t, learning_rate=1e-3, gradient_accumulation_steps=2)
    feats = torch.randn(2, 80, 3000, device=dev)
    batches = []
    for seed in (3, 4, 5):
        dec, lab = L.collate(L.synthetic_label_lists(2, seed=seed, max_len=64))
        batches.append({"input_features": feats, "decoder_input_ids": torch.from_numpy(dec).to(dev),
                        "labels": torch.from_numpy(lab).to(dev)})
    tr.train_step(batches[0])
    tr.train_step(batches[1])
    assert tr.step == 1 and tr.micro == 0
    before = s.store.p32.clone()
    tr.train_step(batches[2], end_of_dataloader=True)
    assert tr.step == 2 and tr.micro == 0
    assert not torch.equal(before, s.store.p32)


def test_entry_point_float32_dtype(tmp_path):
    """--dtype float32 (the reference's default: mixed_precision="no", teacher in fp32,
    run_distillation.py:815-823) trains and evaluates on the fp32 arithmetic path; --dtype float16
    (mixed_precision="fp16": fp16 teacher, fp16 autocast, dynamic loss scaling) trains and evaluates too."""
    from tw.run_distillation import main
    teacher, student = _model_dirs(str(tmp_path))
    man = _corpus(str(tmp_path / "corpus"))
    out = str(tmp_path / "out32")
    common = ["--model_name_or_path", student, "--teacher_model_name_or_path", teacher, "--output_dir", out,
              "--train_dataset_manifest", man, "--eval_dataset_manifest", man, "--per_device_train_batch_size", "2",
              "--per_device_eval_batch_size", "3", "--learning_rate", "1e-4", "--save_steps", "100",
              "--logging_steps", "1", "--freeze_encoder", "True", "--language", "zh", "--do_eval", "True",
              "--predict_with_generate", "True", "--max_label_length", "64", "--byte_level_text_tokenizer", "True",
              "--dataloader_num_workers", "2", "--streaming", "False", "--max_steps", "2", "--eval_steps", "2"]
    res = main(common + ["--dtype", "float32"])
    assert [h["step"] for h in res["train"]] == [1, 2]
    assert all(np.isfinite(h["loss"]) for h in res["train"]) and np.isfinite(res["eval"][0]["loss"])
    res16 = main(common + ["--dtype", "float16", "--output_dir", str(tmp_path / "out16")])
    assert [h["step"] for h in res16["train"]] == [1, 2]
    assert all(np.isfinite(h["loss"]) for h in res16["train"]) and np.isfinite(res16["eval"][0]["loss"])
    # same data and weights: the fp16 run's first loss is the fp32 run's up to fp16 rounding
    assert abs(res16["train"][0]["loss"] - res["train"][0]["loss"]) <= 2e-2 * abs(res["train"][0]["loss"])
