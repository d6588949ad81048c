"""Entry point with the reference's CLI (training/run_distillation.py, argument dataclasses :81-434 +
Seq2SeqTrainingArguments), driving the MI355X engine end to end:

  data      tw.dataset (NTU-COOL manifest + 5-line transcripts, per-rank micro-batches, GPU log-mel)
  step      tw.distill.DistillationTrainer.train_step   (:1507-1552, :1662-1670)
  eval      eval_step + generate_step + compute_metrics  (:1554-1584, :1366-1387, :1709-1800)
  state     accelerate save_state layout, checkpoint-{step}-epoch-{epoch}, rotation, resume + skip
            (:730-774, :1603-1660, :1685-1699), final save_pretrained (:1814-1818)

Launch like the reference (`accelerate launch` → `torchrun`): one process per GPU, RANK / WORLD_SIZE /
LOCAL_RANK from the environment, backend nccl (= RCCL over xGMI) for the gradient exchange.
Flags that only drive subsystems outside the hot path (wandb, push_to_hub, HF-hub datasets, prefiltering)
are accepted and ignored.  Eval data: the reference loads HF-hub datasets by name (unavailable offline);
here `--eval_dataset_manifest` takes a manifest in the same format as the training one.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from typing import Optional

import numpy as np
import torch


def _bool(s):
    return str(s).lower() in ("1", "true", "yes", "y")


def build_parser():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    a = ap.add_argument
    # ModelArguments
    a("--model_name_or_path", required=True)
    a("--teacher_model_name_or_path", required=True)
    a("--tokenizer_name", default=None)
    a("--attn_implementation", default=None)
    a("--mix_lang_emb", type=_bool, default=False)
    a("--dtype", default="float32", help="teacher / compute dtype: bfloat16 | float16 | float32")
    # DataTrainingArguments
    a("--train_dataset_manifest", default=None)
    a("--train_dataset_root", default=None)
    a("--eval_dataset_manifest", default=None)
    a("--eval_dataset_root", default=None)
    a("--max_eval_samples", type=int, default=None)
    a("--max_label_length", type=int, default=448)
    a("--timestamp_probability", type=float, default=0.2)
    a("--condition_on_prev_probability", type=float, default=0.2)
    a("--return_timestamps", type=_bool, default=False)
    a("--language", default=None)
    a("--task", default="transcribe")
    a("--freeze_encoder", type=_bool, default=False)
    a("--freeze_decoder", type=_bool, default=False)
    a("--freeze_embed_positions", type=_bool, default=False)
    a("--temperature", type=float, default=2.0)
    a("--kl_weight", type=float, default=1.0)
    a("--save_valid_best", type=_bool, default=True)
    # Seq2SeqTrainingArguments (the subset the loop reads)
    a("--output_dir", required=True)
    a("--do_train", type=_bool, default=True)
    a("--do_eval", type=_bool, default=False)
    a("--predict_with_generate", type=_bool, default=False)
    a("--generation_num_beams", type=int, default=None)
    a("--per_device_train_batch_size", type=int, default=8)
    a("--per_device_eval_batch_size", type=int, default=8)
    a("--gradient_accumulation_steps", type=int, default=1)
    a("--learning_rate", type=float, default=5e-5)
    a("--weight_decay", type=float, default=0.0)
    a("--adam_beta1", type=float, default=0.9)
    a("--adam_beta2", type=float, default=0.999)
    a("--adam_epsilon", type=float, default=1e-8)
    a("--max_grad_norm", type=float, default=1.0)
    a("--lr_scheduler_type", default="linear")
    a("--warmup_steps", type=int, default=0)
    a("--max_steps", type=int, default=-1)
    a("--num_train_epochs", type=float, default=3.0)
    a("--logging_steps", type=int, default=25)
    a("--save_steps", type=int, default=500)
    a("--eval_steps", type=int, default=None)
    a("--save_total_limit", type=int, default=None)
    a("--resume_from_checkpoint", default=None)
    a("--seed", type=int, default=42)
    a("--dataloader_num_workers", type=int, default=4)
    a("--streaming", type=_bool, default=True)
    # accepted for CLI compatibility, no effect here
    for flag in ("--wandb_project", "--wandb_name", "--wandb_dir", "--push_to_hub", "--overwrite_output_dir",
                 "--is_prefiltered", "--skip_audio_length_filtering", "--gradient_checkpointing", "--bf16", "--fp16",
                 "--preprocessing_num_workers", "--report_to", "--use_pseudo_labels", "--text_column_name",
                 "--eval_text_column_name", "--train_dataset_name", "--eval_dataset_name", "--cache_dir",
                 "--dataset_cache_dir", "--wer_threshold", "--dataloader_prefetch_factor", "--ddp_timeout"):
        a(flag, default=None)
    # engine-specific
    a("--byte_level_text_tokenizer", type=_bool, default=False,
      help="tokenize transcript text bytes (testing without tokenizer files)")
    return ap


def load_tokenizer(args):
    """The reference's WhisperTokenizerFast (+1501 timestamp tokens) when its files exist in the model
    directory; else the special-token adapter over a byte-level text encoder (tests only)."""
    from .dataset import WhisperTokenizerAdapter
    path = args.tokenizer_name or args.model_name_or_path
    if not args.byte_level_text_tokenizer:
        from transformers import AddedToken, WhisperTokenizerFast
        tok = WhisperTokenizerFast.from_pretrained(path)
        tok.add_tokens([AddedToken("<|%.2f|>" % (i * 0.02), lstrip=False, rstrip=False) for i in range(1501)])
        if args.language is not None:
            tok.set_prefix_tokens(language=args.language, task=args.task,
                                  predict_timestamps=args.timestamp_probability > 0)
        return tok
    return WhisperTokenizerAdapter(lambda s: list(s.encode("utf-8")), language=args.language, task=args.task,
                                   predict_timestamps=args.timestamp_probability > 0,
                                   text_decoder=lambda ids: bytes(i for i in ids if i < 256).decode("utf-8", "ignore"))


def _dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    if world > 1 and not torch.distributed.is_initialized():
        torch.distributed.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    return rank, world


def _mean_over_ranks(metrics: dict, world: int) -> dict:
    keys = sorted(metrics)
    v = torch.stack([metrics[k].float().reshape(()) for k in keys])
    if world > 1:
        torch.distributed.all_reduce(v)
        v /= world
    return {k: float(x) for k, x in zip(keys, v.tolist())}


def gather_eval_rows(rows, world: int):
    """[(batch index, preds, labels)] of every rank -> flat preds / labels in gather_for_metrics order
    (batch-major, then rank)."""
    gathered = [rows]
    if world > 1:
        gathered = [None] * world
        torch.distributed.all_gather_object(gathered, rows)
    merged = sorted(((bi, r, p, l) for r, rk in enumerate(gathered) for bi, p, l in rk), key=lambda x: (x[0], x[1]))
    preds = [x for _, _, p, _ in merged for x in p]
    labels = [x for _, _, _, l in merged for x in l]
    return preds, labels


def evaluate(trainer, feed, tokenizer, gen_kwargs: dict, predict_with_generate: bool, world: int,
             return_timestamps: bool = False):
    """The eval block of the loop (:1709-1800): mean of the eval_step metrics over every (batch, rank)
    scalar (torch.mean of the gathered per-rank scalars), greedy generation of every batch, MER (x100)
    on the decoded strings of all ranks.  Predictions / labels follow gather_for_metrics: gathered
    batch by batch in rank order, the wrap-around duplicates of the last (even_batches) group dropped
    (batch["n_real"] from DataFeed), so each eval item is scored exactly once."""
    from .evaluation import compute_metrics
    sums, n = None, 0
    rows = []                      # (batch index, preds, labels) of this rank, duplicates dropped
    for bi, batch in enumerate(feed):
        m = trainer.eval_step(batch)
        v = torch.stack([m["loss"], m["ce_loss"], m["kl_loss"]]).float()
        sums = v if sums is None else sums + v
        n += 1
        if predict_with_generate:
            keep = int(batch.get("n_real", batch["labels"].shape[0]))
            ids = trainer.s.generate(batch["input_features"], **gen_kwargs)
            rows.append((bi, [r.tolist() for r in ids[:keep].cpu()], [r.tolist() for r in batch["labels"][:keep].cpu()]))
    if world > 1:
        torch.distributed.all_reduce(sums)
        cnt = torch.tensor([float(n)], device=sums.device)
        torch.distributed.all_reduce(cnt)
        n = int(cnt.item())
    preds, labels = gather_eval_rows(rows, world) if predict_with_generate else ([], [])
    out = {k: float(x) / max(n, 1) for k, x in zip(("loss", "ce_loss", "kl_loss"), sums.tolist())} if sums is not None else {}
    if predict_with_generate and preds:
        wer, *_ = compute_metrics(preds, labels, tokenizer, return_timestamps=return_timestamps)
        out.update(wer)
    return out


def teacher_dtype(dtype: str):
    """--dtype -> teacher weight dtype (run_distillation.py:815-823).  bfloat16 = bf16 autocast
    (mixed_precision="bf16"); float16 = fp16 autocast with the dynamic loss scaler (mixed_precision="fp16",
    fp16 teacher); float32 = mixed_precision="no" (fp32 arithmetic end to end, the reference's default)."""
    if dtype == "bfloat16":
        return torch.bfloat16
    if dtype == "float16":
        return torch.float16
    if dtype == "float32":
        from .modeling import fp32_compute_supported
        if not fp32_compute_supported():
            raise NotImplementedError("--dtype float32 (mixed_precision='no') needs the fp32 arithmetic path")
        return torch.float32
    raise ValueError(f"--dtype {dtype}: one of float32, float16, bfloat16 (run_distillation.py:417-424)")


def load_models(args, device, tokenizer=None):
    """Teacher (in --dtype) and fp32-master student, as run_distillation.py:1009-1031 loads them; with
    --mix_lang_emb only the TEACHER is mixed (:1019-1020) — the student's <|zh|> row was mixed once at
    creation (create_student_model.py:124-125)."""
    from .modeling import WhisperForConditionalGeneration
    from .student import mix_language_embeddings
    # mixed_precision "no" / "fp16" / "bf16" (:815-823)
    compute = {"float32": "fp32", "float16": "fp16"}.get(args.dtype, "bf16")
    teacher = WhisperForConditionalGeneration.from_pretrained(args.teacher_model_name_or_path,
                                                              torch_dtype=teacher_dtype(args.dtype), device=device,
                                                              compute=compute)
    student = WhisperForConditionalGeneration.from_pretrained(args.model_name_or_path, device=device, compute=compute)
    if args.mix_lang_emb:
        mix_language_embeddings(teacher, tokenizer if hasattr(tokenizer, "convert_tokens_to_ids") else None,
                                languages=["zh", "en"])
    return teacher, student


def main(argv=None):
    from .checkpoint import (checkpoint_name, get_last_checkpoint, parse_checkpoint, resume_skip_batches,
                             rotate_checkpoints)
    from .dataset import CoolDataset, DataFeed
    from .distill import DistillationTrainer
    from .modeling import WhisperForConditionalGeneration
    from .student import mix_language_embeddings

    args = build_parser().parse_args(argv)
    rank, world = _dist()
    dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(args.seed)
    os.makedirs(args.output_dir, exist_ok=True)
    tokenizer = load_tokenizer(args)
    teacher, student = load_models(args, dev, tokenizer)
    trainer = DistillationTrainer(
        student, teacher, temperature=args.temperature, kl_weight=args.kl_weight, learning_rate=args.learning_rate,
        adam_beta1=args.adam_beta1, adam_beta2=args.adam_beta2, adam_epsilon=args.adam_epsilon,
        weight_decay=args.weight_decay, max_grad_norm=args.max_grad_norm, warmup_steps=args.warmup_steps,
        lr_scheduler_type=args.lr_scheduler_type, max_steps=max(args.max_steps, 0),
        gradient_accumulation_steps=args.gradient_accumulation_steps, freeze_encoder=args.freeze_encoder,
        freeze_decoder=args.freeze_decoder, freeze_embed_positions=args.freeze_embed_positions,
        process_group=torch.distributed.group.WORLD if world > 1 else None)
    gen_kwargs = {"max_length": args.max_label_length, "num_beams": args.generation_num_beams or 1,
                  "return_timestamps": args.return_timestamps and args.timestamp_probability > 0}
    if args.language is not None:
        gen_kwargs.update(language=args.language, task=args.task)
    prep = dict(timestamp_probability=args.timestamp_probability,
                condition_on_prev_probability=args.condition_on_prev_probability,
                max_label_length=args.max_label_length)

    train_ds = CoolDataset(args.train_dataset_manifest, args.train_dataset_root) if args.do_train else None
    eval_ds = CoolDataset(args.eval_dataset_manifest, args.eval_dataset_root) if args.eval_dataset_manifest else None
    accum = args.gradient_accumulation_steps
    steps_per_epoch = (len(train_ds) // (args.per_device_train_batch_size * world * accum)) if train_ds else 0
    total = args.max_steps if args.max_steps > 0 else int(steps_per_epoch * args.num_train_epochs)
    trainer.max_steps = total
    eval_steps = args.eval_steps or steps_per_epoch or total

    cur_step, epochs_trained, skip = 0, 0, 0
    ckpt = args.resume_from_checkpoint or get_last_checkpoint(args.output_dir)
    if ckpt:
        trainer.load_state(ckpt)
        cur_step, epochs_trained = parse_checkpoint(ckpt)
        # None: the reference re-shuffles with the same seed and restarts the resumed epoch from its
        # first batch (:1629-1640; set_epoch(epoch) makes that the same order again)
        skip = resume_skip_batches(cur_step, epochs_trained, steps_per_epoch, accum, args.streaming,
                                   args.max_steps) or 0
    best_wer, log_every, t0 = 100.0, max(1, args.logging_steps), time.time()
    history, evals = [], []
    epoch = epochs_trained
    while train_ds is not None and cur_step < total:
        feed = DataFeed(train_ds, tokenizer, args.per_device_train_batch_size, rank=rank, world=world, device=dev,
                        seed=args.seed, epoch=epoch, skip_batches=skip, workers=args.dataloader_num_workers, **prep)
        skip = 0
        n_batches = len(feed)
        for bi, batch in enumerate(feed):
            m = trainer.train_step(batch, temperature=args.temperature, end_of_dataloader=bi + 1 == n_batches)
            if trainer.micro != 0:
                continue                                     # accumulating
            cur_step += 1
            if cur_step % log_every == 0:
                mm = _mean_over_ranks(m, world)
                mm.update(step=cur_step, epoch=epoch, lr=trainer.lr_at(trainer.step), time=time.time() - t0)
                history.append(mm)
                if rank == 0:
                    print(json.dumps({"train": mm}), flush=True)
            if cur_step % args.save_steps == 0 or cur_step == total:
                d = os.path.join(args.output_dir, checkpoint_name(cur_step, epoch))
                trainer.save_state(d, rank=rank)
                if world > 1:
                    torch.distributed.barrier()
                if rank == 0:
                    rotate_checkpoints(args.save_total_limit, args.output_dir)
            if args.do_eval and eval_ds is not None and (cur_step % eval_steps == 0 or cur_step == total):
                ef = DataFeed(eval_ds, tokenizer, args.per_device_eval_batch_size, rank=rank, world=world, device=dev,
                              seed=args.seed, shuffle=False, timestamp_probability=0.0,
                              condition_on_prev_probability=0.0, max_label_length=args.max_label_length)
                em = evaluate(trainer, ef, tokenizer, gen_kwargs, args.predict_with_generate, world,
                              gen_kwargs["return_timestamps"])
                em.update(step=cur_step)
                evals.append(em)
                if rank == 0:
                    print(json.dumps({"eval": em}), flush=True)
                if args.save_valid_best and "wer" in em and em["wer"] < best_wer:
                    best_wer = em["wer"]
                    d = os.path.join(args.output_dir, f"best-checkpoint-epoch-{epoch}")
                    trainer.save_state(d, rank=rank)
                    if rank == 0:
                        with open(os.path.join(d, "best_steps.txt"), "w") as f:
                            f.write(f"step: {cur_step}, wer: {best_wer}, epoch: {epoch}")
            if cur_step >= total:
                break
        epoch += 1
    trainer.flush()                                          # a deferred last update (DP overlap)
    if rank == 0:
        student.save_pretrained(args.output_dir)
    if world > 1:
        torch.distributed.barrier()
    return {"train": history, "eval": evals}


if __name__ == "__main__":
    main()
