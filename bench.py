#!/usr/bin/env python
"""Distillation-step throughput on MI355X (BASELINE.json metric: distillation utt/s on 30 s
clips at 1/2/4/8 GPUs; teacher-fwd ms/clip).

Workload (default, BASELINE config 3): 2-decoder-layer distil-whisper student made by the
create_student_model layer map from a large-v2 teacher, frozen shared encoder, batch 64 clips per
GPU, bf16 autocast semantics, full step = GPU log-mel + student fwd + teacher fwd + fused KL/CE +
student bwd + (DP all-reduce) + clip + AdamW.  `--config c2` runs config 2 (whisper-small student,
trainable encoder, full large-v2 teacher forward, B = 32).  `--config c4` is the pseudo-labelling
path (initial_inference.py / run_pseudo_labelling.py:917-922): large-v2 batched greedy transcription of
512 synthetic 30 s clips (GPU log-mel + encoder + KV-cache decode, 224 new tokens per clip: eos is
suppressed so the work is fixed), a step = one batch of --batch clips.  `--config c5` is
the long-form eval path (run_eval.py:659-685): one 30-minute synthetic recording, long-form log-mel,
sequential 30 s windows with timestamp tokens, cross-attention K/V projected once per window and reused
by every step (a step = the whole recording; value = audio seconds per wall second).  Random-init weights of the real
architectures (no checkpoints offline) and synthetic 30 s / 16 kHz sine clips + synthetic labels
(SURVEY.md §8(d)); inputs are resident in HBM before the timed region.

One process per GPU (torch.distributed.run); each rank processes its own 64 clips (weak scaling),
gradients are averaged with an RCCL all-reduce; rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "taiwan-whisper_amd"))

import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip table)
PEAK_HBM_GBS = 8000.0


def _flops_per_clip(cfg_s, cfg_t, share, T_dec=447, T_enc=1500):
    """Algorithmic FLOPs of one distillation step per clip (SURVEY.md §8(d) formula:
    2*MAC of every GEMM + QK^T/PV at full size; no recompute)."""
    def fwd(c, enc=True):
        d, V, fe, fd = c.d_model, c.vocab_size, c.encoder_ffn_dim, c.decoder_ffn_dim
        conv = 2 * (2 * T_enc) * (c.num_mel_bins * 3) * d + 2 * T_enc * (3 * d) * d
        el = 2 * T_enc * d * 4 * d + 2 * 2 * T_enc * d * fe + 2 * 2 * T_enc * T_enc * d
        dl = (2 * T_dec * d * 4 * d + 2 * 2 * T_dec * T_dec * d + 2 * T_dec * d * 2 * d + 2 * T_enc * d * 2 * d
              + 2 * 2 * T_dec * T_enc * d + 2 * 2 * T_dec * d * fd)
        e = conv + c.encoder_layers * el
        return (e if enc else 0), c.decoder_layers * dl + 2 * T_dec * d * V
    se, sd = fwd(cfg_s)
    te, td = fwd(cfg_t)
    if share:     # frozen shared encoder: fwd once; student decoder fwd+bwd = 3x; teacher decoder fwd
        return se + 3 * sd + td
    return 3 * (se + sd) + te + td


def make_models(args, device):
    from tw.config import WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration, random_init_
    from tw.student import student_from_teacher
    large = dict(d_model=1280, encoder_layers=32, decoder_layers=32, encoder_attention_heads=20,
                 decoder_attention_heads=20, encoder_ffn_dim=5120, decoder_ffn_dim=5120)
    small = dict(d_model=768, encoder_layers=12, decoder_layers=12, encoder_attention_heads=12,
                 decoder_attention_heads=12, encoder_ffn_dim=3072, decoder_ffn_dim=3072)
    tcfg = WhisperConfig(**large)
    # --dtype bf16 (every reference launcher) or fp16 (--dtype float16: fp16 teacher, fp16-autocast student + loss
    # scaler, run_distillation.py:815-817)
    tdt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    if args.config == "c3":
        t32 = random_init_(WhisperForConditionalGeneration(tcfg, dtype=torch.float32, device=device), seed=0)
        student, _, _ = student_from_teacher(t32, encoder_layers=32, decoder_layers=2)
        teacher = WhisperForConditionalGeneration(tcfg, dtype=tdt, device=device)
        if tdt == torch.float16:
            teacher.store.p16.copy_(t32.store.p32)   # torch_dtype=fp16 teacher
        else:
            teacher.store.p16.copy_(t32.store.p16)   # torch_dtype=bf16 teacher (run_distillation.py:1011-1018)
        teacher._refresh_ln32()
        del t32
        freeze_encoder = True
    else:
        teacher = random_init_(WhisperForConditionalGeneration(tcfg, dtype=tdt, device=device), seed=0)
        student = random_init_(WhisperForConditionalGeneration(WhisperConfig(**small), dtype=torch.float32,
                                                               device=device), seed=1)
        freeze_encoder = False
    if args.dtype == "fp16":
        student.set_compute("fp16")
    torch.cuda.empty_cache()
    return student, teacher, freeze_encoder


def make_batches(args, device, rank, nb=2):
    from tw.data import DataCollatorSpeechSeq2SeqWithPadding, synthetic_audio, synthetic_label_lists
    coll = DataCollatorSpeechSeq2SeqWithPadding(max_target_length=448)
    out = []
    for i in range(nb):
        seed = 1000 * rank + i
        wav = synthetic_audio(args.batch, seed=seed, device=device)
        dec, lab = coll.collate_labels(synthetic_label_lists(args.batch, seed=seed))
        out.append((wav, dec.to(device), lab.to(device)))
    return out


def cpu_baseline(seconds_budget=20.0):
    """Oracle (CPU restatement of the reference train_step, fp32, AdamW) on config 1:
    whisper-tiny student + tiny teacher, B = 2 synthetic 30 s clips, host cores."""
    sys.path.insert(0, REPO)
    import numpy as np
    from oracle import distill_ref, labels as L, logmel
    from oracle.weights import CONFIGS, make_weights
    from oracle.whisper_ref import Ref, to_torch
    # the job's CPU share: OMP_NUM_THREADS where the launcher sets it (the GPU box gives a 1-GPU job 16 threads of a
    # much larger host; only the first field of a nested value such as "16,1" counts), else the CPUs this process may
    # run on, capped at 16 so that `cores` stays comparable across hosts and rounds
    host = os.cpu_count() or 1
    omp = (os.environ.get("OMP_NUM_THREADS") or "").split(",")[0].strip()
    threads = int(omp) if omp.isdigit() and int(omp) > 0 else min(16, len(os.sched_getaffinity(0)) or host)
    torch.set_num_threads(threads)
    cfg = CONFIGS["tiny"]
    ps = to_torch(make_weights(cfg, 1))
    pt = to_torch(make_weights(cfg, 2))
    names = [n for n in ps if not n.startswith("model.encoder") and "embed_positions" not in n]
    for n in names:
        ps[n].requires_grad_(True)
    S, T = Ref(cfg, ps), Ref(cfg, pt)
    B = 2
    feats = torch.from_numpy(logmel.log_mel_batch([logmel.synthetic_clip(i) for i in range(B)]))
    dec, lab = L.collate(L.synthetic_label_lists(B, seed=0))
    dec, lab = torch.from_numpy(dec), torch.from_numpy(lab)
    opt = None
    times = []
    t_start = time.time()
    while True:
        t0 = time.time()
        # feature extraction is part of the reference step (dataloader workers, :1217)
        feats = torch.from_numpy(logmel.log_mel_batch([logmel.synthetic_clip(i) for i in range(B)]))
        for n in names:
            ps[n].grad = None
        distill_ref.train_step(S, T, feats, dec, lab, share_hidden_states=True)
        _, opt = distill_ref.optimizer_step(ps, names, lr=1e-4, state=opt)
        times.append(time.time() - t0)
        if time.time() - t_start > seconds_budget or len(times) >= 12:
            break
    steady = times[1:] if len(times) > 1 else times
    per = sum(steady) / len(steady)
    return dict(value=round(B / per, 4), unit="utt/s", cores=threads, host_cores=host,
                cores_note=f"{threads} threads = this job's CPU share (OMP_NUM_THREADS / affinity) of a host with "
                           f"{host} logical CPUs", kind="port",
                sample=f"config 1 (tiny<-tiny, B=2, fp32, frozen shared encoder, CPU log-mel + train_step + "
                       f"AdamW) via oracle/distill_ref.py, {len(steady)} steady steps of {len(times)}")


PMC_FILE = "profiles/pmc_latest.json"
MFMA_FILE = "profiles/mfma_latest.json"


def _committed(path):
    """(summary dict, source note) of a committed rocprofv3 --pmc summary: the file's own `source` field names the
    command, tree and box it came from (PMC counters need their own profiler passes, so they are never this run's)."""
    p = os.path.join(REPO, path)
    if not os.path.exists(p):
        return {}, None
    with open(p) as f:
        d = json.load(f)
    return d, f"{path}: {d.get('source', 'source not recorded')}"


def load_pmc(kernel_family):
    """Per-launch HBM bytes of the dominant kernel from the committed rocprofv3 --pmc summary, and its source."""
    d, src = _committed(PMC_FILE)
    return d.get(kernel_family, {}).get("hbm_bytes_per_launch"), src


def decode_bytes_per_step(cfg, B, t_avg, Tk=1500, elem=2):
    """Algorithmic HBM bytes of one greedy decode step over B rows: every decoder weight once (the
    per-layer Linears + LayerNorms, the tied head over the padded vocabulary), the cross-attention
    K/V of every clip and layer, and the self-attention K/V rows 0..t (t_avg = mean step index)."""
    d, f, L, Vp = cfg.d_model, cfg.decoder_ffn_dim, cfg.decoder_layers, (cfg.vocab_size + 63) // 64 * 64
    weights = L * (6 * d * d + 2 * d * f) * elem + Vp * d * elem
    cross = L * B * Tk * 2 * d * elem
    self_kv = L * B * t_avg * 2 * d * elem
    return weights + cross + self_kv


def _heartbeat(tag, every=30.0):
    """Print a progress line to stderr every `every` seconds while a long decode runs (the c5 step with the
    reference's fallback kwargs is minutes long; a silent process looks hung to the GPU-box watchdog)."""
    import threading
    t0 = time.time()
    stop = threading.Event()

    def loop():
        while not stop.wait(every):
            print(f"[bench {tag}] running, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=loop, daemon=True).start()
    return stop


def run_decode(args, device, rank, world, pg):
    """c4 (batched greedy pseudo-labelling) and c5 (long-form eval) on large-v2 (random-init bf16:
    the reference runs these in the checkpoint's dtype under its fp16/bf16 flag)."""
    from tw.config import LARGE_V2_SUPPRESS, MODEL_DIMS, GenerationConfig, WhisperConfig
    from tw.data import synthetic_audio
    from tw.feature_extraction import WhisperFeatureExtractor
    from tw.modeling import WhisperForConditionalGeneration, random_init_
    from tw.profiling import KernelTimer
    cfg = WhisperConfig(**MODEL_DIMS["large-v2"])
    hb = _heartbeat(args.config)
    # --dtype fp16 (default): the reference's decode arithmetic (run_eval.py:99 --dtype float16, :500-509;
    # run_pseudo_labelling.py:461-463 via run-pseudo-labelling.sh:30); bf16: the autocast-style bf16 model
    dt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    m = random_init_(WhisperForConditionalGeneration(cfg, dtype=dt, device=device), seed=0)
    fe = WhisperFeatureExtractor(device=device)
    c4 = args.config == "c4"
    # c4: eos suppressed -> every clip decodes exactly --new-tokens (SURVEY.md §8d fixed work)
    m.generation_config = GenerationConfig(suppress_tokens=LARGE_V2_SUPPRESS + ([50257] if c4 else []),
                                           begin_suppress_tokens=[220, 50257], lang_to_id={"<|zh|>": 50260},
                                           max_initial_timestamp_index=50)   # large-v2 generation_config.json
    if c4:
        kw = dict(language="zh", task="transcribe", max_new_tokens=args.new_tokens)
    else:
        # run_eval.py:637-642 gen_kwargs (generation_max_length 256, :210-211) merged with the long-form
        # kwargs of :659-665 at their defaults (:148-176: temperature fallback on, compression 1.35, log-prob
        # -1.0, no-speech 0.6, no conditioning) for every input longer than 30 s (:673-676).
        # --longform-kwargs none: greedy windows only (the round-2 workload, for comparison).
        kw = dict(language="zh", task="transcribe", max_length=256)
        if args.longform_kwargs == "ref":
            kw.update(condition_on_prev_tokens=False, compression_ratio_threshold=1.35,
                      temperature=(0.0, 0.2, 0.4, 0.6, 0.8, 1.0), logprob_threshold=-1.0, no_speech_threshold=0.6)
    if c4:
        wavs = [synthetic_audio(args.batch, seed=1000 * rank + i, device=device) for i in range(2)]

        def step(i):
            mel, _ = fe.extract(wavs[i % 2], want_conv_input=False)
            return m.generate(mel, **kw)
        units_per_step, unit = args.batch, "utt/s"
    else:
        # --batch N: N recordings in ONE generate call, kept together window after window (HF's batched long-form,
        # run_eval.py:667-681 with inner_batch_size recordings)
        n = int(args.seconds * 16000)
        wav = synthetic_audio(args.batch, seed=1000 * rank, seconds=args.seconds, device=device, length=None)
        mel_long, _ = fe.extract(wav, want_conv_input=False)           # features prepared outside the timed
        mask = torch.ones(args.batch, n // 160, dtype=torch.int32, device=device)   # region, as run_eval.py:567-589
        trace = []

        def step(i):
            trace.clear()
            return m.generate(mel_long, attention_mask=mask, return_timestamps=True, _trace=trace, **kw)
        units_per_step, unit = args.seconds * args.batch, "audio s/s"
    for i in range(args.warmup):
        if c4:
            step(i)
        else:      # warm-up on a 65 s prefix (the kernels and graph capture; not the full recording)
            m.generate(mel_long[:, :, :6500], attention_mask=mask[:, :6500], return_timestamps=True, **kw)
            trace.clear()
    torch.cuda.synchronize()
    if pg is not None:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = step(i)
    torch.cuda.synchronize()
    if pg is not None:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    trace_last = list(trace) if not c4 else None
    if pg is not None:
        torch.distributed.all_reduce(elapsed, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    if c4:
        dec_steps = args.steps * (out.shape[1] + 3)                 # prompt prefill (3) + generated columns
        B, t_avg = args.batch, 4 + out.shape[1] / 2
    else:
        # row-steps (one decoder step of one row); with --batch N the rows of a batch share each launch
        dec_steps = args.steps * sum(len(t["raw"]) + len(t["prompt"]) - 1 for t in trace_last)
        B, t_avg = 1, 4 + sum(len(t["raw"]) for t in trace_last) / max(1, 2 * len(trace_last))
    ms_dec = elapsed / dec_steps * 1e3
    step_bytes = decode_bytes_per_step(cfg, B, t_avg)
    # dominant kernel (cross-attention over the encoder K/V, the largest per-step read): per-launch HIP
    # events over an eager (non-graph) decode of the same batch shape, 16 steps
    timer = KernelTimer("decode_attn_cross")
    with timer:
        if c4:
            mel, _ = fe.extract(wavs[0], want_conv_input=False)
            m.generate(mel, use_graph=False, language="zh", task="transcribe", max_new_tokens=16)
        else:
            m.generate(mel_long[:, :, :3000], use_graph=False, return_timestamps=True, language="zh",
                       task="transcribe", max_new_tokens=16)
            trace.clear()
    ks = timer.summary()
    if rank == 0:
        value = units_per_step * args.steps * world / elapsed
        roof = None
        if ks is not None:
            achieved = ks["rate"] / 1e9
            roof = dict(bound="hbm", achieved=round(achieved, 1), peak=PEAK_HBM_GBS, unit="GB/s",
                        frac=round(achieved / PEAK_HBM_GBS, 4), traffic=None,
                        kernel="decode_attn_u2/u4_kernel (cross-attention over the per-layer encoder K/V cache)",
                        bytes_per_launch=int(ks["avg_work"]), avg_launch_ms=round(ks["avg_ms"], 5),
                        launches_timed=ks["launches"])
        out_d = {
            "metric": ("pseudo-labelling greedy transcription utterances/sec (30 s clips)" if c4 else
                       "long-form transcription speed (audio seconds per wall second)"),
            "value": round(value, 3), "unit": unit, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (sines + noise, random-init large-v2 weights)" + (
                "; eos suppressed -> fixed tokens per clip" if c4 else ""),
            "config": {"workload": (f"c4: whisper-large-v2 batched greedy, {args.batch} x 30 s clips per step, "
                                    f"{args.new_tokens} new tokens" if c4 else
                                    f"c5: whisper-large-v2 long-form, {args.batch} x {args.seconds:.0f} s recording(s) "
                                    f"in one generate call, timestamps, max_length 256 per window, long-form kwargs "
                                    f"{args.longform_kwargs}"),
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch, "parallelism":
                       f"replicas{world}"},
            "decode_steps": dec_steps, "ms_per_decode_step": round(ms_dec, 4),
            # batch-1 steps only: a row-step of a batched decode shares its weight reads with the batch's other rows
            "decode_step_hbm_frac": (round(step_bytes / (ms_dec * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
                                     if c4 or args.batch == 1 else None),
            "roofline": roof,
            "cpu_baseline": None,
        }
        if not c4:
            wins = {}
            for t in trace_last:
                wins.setdefault((t["b"], t["seek"]), []).append(t)
            decodes = len(trace_last)
            skipped = sum(1 for v in wins.values() if v[-1].get("skip"))
            out_d["windows"] = len(wins)
            out_d["decodes"] = decodes
            out_d["fallback_decodes_per_window"] = round((decodes - len(wins)) / max(1, len(wins)), 3)
            out_d["windows_all_temperatures_failed"] = sum(1 for v in wins.values() if v[-1].get("needs_fallback"))
            out_d["windows_skipped_no_speech"] = skipped
            out_d["gate_ms_per_step"] = round(sum(t.get("gate_ms", 0.0) for t in trace_last), 3)
            out_d["longform_kwargs"] = (
                "run_eval.py:659-665 defaults: temperature (0.0,0.2,...,1.0), compression_ratio 1.35, "
                "logprob -1.0, no_speech 0.6, max_length 256" if args.longform_kwargs == "ref" else
                "none (greedy windows only), max_length 256")
            if args.longform_kwargs == "ref" and decodes >= 5 * len(wins):
                out_d["note"] = ("random-init weights: the average log-prob of every window is far below -1.0, so "
                                 "HF's fallback re-decodes each window at all 6 temperatures (the work of a real "
                                 "checkpoint is mostly the T=0 pass); --longform-kwargs none times greedy windows")
            out_d["real_time_factor"] = round(elapsed / args.steps / args.seconds, 5)
        print(json.dumps(out_d), flush=True)
    hb.set()
    if pg is not None:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def exchange_summary(ev, log, steps, t_rank, pg, world, device):
    """The `distributed` object of the JSON line (collective over the ranks: every rank calls it).
    ev: the trainer's exchange_events, (start, layers done, tail done) events per timed exchange wait on the compute
    stream (anything with .elapsed_time); log: its exchange_log, (bytes, tail) per all-reduced bucket; t_rank: this
    rank's own time for the timed steps, taken before the closing barrier."""
    if pg is None:
        return dict(backend=None, world_size=1, exchange=None)
    # compute-stream time between reaching the gradient-exchange wait and passing it (the all-reduce time the step
    # does not hide), per timed step: the buckets launched per finished layer during the backward, then the tail
    # launched after it (tied embedding + final LayerNorm, final only after the embedding backward)
    layers_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / steps
    tail_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / steps
    backend = torch.distributed.get_backend(pg)
    per_rank = torch.tensor([t_rank / steps * 1e3, layers_ms + tail_ms], dtype=torch.float64,
                            device="cpu" if backend == "gloo" else device)
    gathered = [torch.zeros_like(per_rank) for _ in range(world)]
    torch.distributed.all_gather(gathered, per_rank, group=pg)
    step_ms = [float(g[0]) for g in gathered]
    exposed = [float(g[1]) for g in gathered]
    nbytes = sum(b for b, _ in log) / steps
    tail_bytes = sum(b for b, t in log if t) / steps
    return dict(backend=backend, world_size=torch.distributed.get_world_size(pg),
                exchange_bytes_per_step=int(nbytes), exchange_tail_bytes_per_step=int(tail_bytes),
                exchange_buckets_per_step=len(log) // steps,
                # a ring all-reduce moves 2 (N - 1) / N of the payload in and out of every GPU
                ring_bytes_per_gpu_per_step=int(2 * (world - 1) / world * nbytes),
                exchange_exposed_ms_per_step=round(layers_ms + tail_ms, 3),
                exchange_exposed_layers_ms_per_step=round(layers_ms, 3),
                exchange_exposed_tail_ms_per_step=round(tail_ms, 3),
                rank_step_ms=[round(x, 3) for x in step_ms],
                rank_step_ms_spread=round(max(step_ms) - min(step_ms), 3),
                rank_exchange_exposed_ms=[round(x, 3) for x in exposed],
                exchange="bucketed async SUM all-reduce of the flat fp32 student gradient, launched per finished "
                         "layer during the backward; clip + AdamW deferred under the next encoder forward")


def load_mfma(workload, family):
    """MFMA-busy fraction (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)) of a kernel family
    from the committed rocprofv3 --pmc summary (tools/pmc_mfma.sh -> profiles/mfma_latest.json)."""
    d, _ = _committed(MFMA_FILE)
    return d.get(workload, {}).get(family, {}).get("mfma_busy_frac")


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`python bench.py --gpus N` outside a launcher: start N ranks (one per GPU) under torch.distributed.run as a
    child process -- before this process makes any GPU call -- and return its exit code.  The same command the
    driver runs: --nnodes 1, --master-addr 127.0.0.1."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    if os.environ.get("TW_BENCH_PRINT_LAUNCH") == "1":          # tests: show the launch, start nothing
        print(json.dumps({"launch": cmd}), flush=True)
        return 0
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default WORLD_SIZE under a launcher, else 1.  Without a launcher, "
                         "N > 1 starts the N ranks itself")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--config", default="c3", choices=["c3", "c2", "c4", "c5"])
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--new-tokens", type=int, default=224, help="c4/c5: new tokens per clip / window")
    ap.add_argument("--seconds", type=float, default=1800.0, help="c5: recording length")
    ap.add_argument("--dtype", default=None, choices=["fp16", "bf16"],
                    help="c4/c5: model dtype (default fp16: the reference's decode call sites default to float16); "
                         "c2/c3: the distillation's mixed precision (default bf16: every reference launcher; fp16 = "
                         "--dtype float16, fp16 autocast + loss scaler)")
    ap.add_argument("--longform-kwargs", default="ref", choices=["ref", "none"],
                    help="c5: run_eval.py:659-665 long-form kwargs (ref) or greedy windows only (none)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-teacher-fwd", action="store_true")
    args = ap.parse_args()
    dflt = {"c3": (64, 10, 3), "c2": (32, 10, 3), "c4": (512, 1, 1), "c5": (1, 1, 1)}[args.config]
    args.batch = dflt[0] if args.batch is None else args.batch
    args.steps = dflt[1] if args.steps is None else args.steps
    args.warmup = dflt[2] if args.warmup is None else args.warmup
    if args.dtype is None:
        args.dtype = "fp16" if args.config in ("c4", "c5") else "bf16"

    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world) if env_world else 1
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks", file=sys.stderr)
        sys.exit(2)
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # TW_BENCH_REHEARSE=1: all ranks on cuda:0 over gloo (multi-rank rehearsal on a 1-GPU box);
    # the real multi-GPU run uses one GPU per rank and RCCL ("nccl").
    rehearse = os.environ.get("TW_BENCH_REHEARSE") == "1"
    # TW_BENCH_FORCE_EXCHANGE=1 (rehearsal of the 8-GPU path on one GPU): a process group even at world 1 and the
    # trainer's DP exchange forced on (per-layer RCCL all-reduces, tail, waits, deferred update), so the line's
    # `distributed` object comes from the backend the 8-GPU node runs
    force_x = os.environ.get("TW_BENCH_FORCE_EXCHANGE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    pg = None
    if force_x and env_world is None:         # not under a launcher: a one-rank rendezvous of our own
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
    if world > 1 or force_x:
        if rehearse:
            torch.distributed.init_process_group("gloo")
        else:
            torch.distributed.init_process_group("nccl", device_id=device)
        pg = torch.distributed.group.WORLD

    if args.config in ("c4", "c5"):
        run_decode(args, device, rank, world, pg)
        return

    from tw.distill import DistillationTrainer
    from tw.feature_extraction import WhisperFeatureExtractor
    from tw.profiling import KernelTimer

    student, teacher, freeze_encoder = make_models(args, device)
    trainer = DistillationTrainer(student, teacher, learning_rate=1e-4, warmup_steps=0,
                                  freeze_encoder=freeze_encoder, process_group=pg, force_exchange=force_x)
    trainer.exchange_events = [] if pg is not None else None     # exposed gradient-exchange waits
    trainer.exchange_log = [] if pg is not None else None        # (bytes, tail) per all-reduced bucket
    fe = WhisperFeatureExtractor(device=device)
    batches = make_batches(args, device, rank)

    def step(i):
        wav, dec, lab = batches[i % len(batches)]
        mel, conv = fe.extract(wav)          # fp16: the trainer casts the log-mel into the fp16 conv input itself
        return trainer.train_step({"conv_input": conv, "input_features": mel, "decoder_input_ids": dec,
                                   "labels": lab})

    for i in range(args.warmup):
        m = step(i)
    trainer.flush()              # the warmup's last update (deferred under DP) stays outside the timed region
    torch.cuda.synchronize()
    if trainer.exchange_events is not None:
        trainer.exchange_events.clear()
        trainer.exchange_log.clear()
    if pg is not None:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    timer = KernelTimer("gemm_nn")
    with timer:
        t0 = time.perf_counter()
        for i in range(args.steps):
            m = step(i)
        trainer.flush()          # ... and the last timed step's update inside it: exactly K updates timed
        torch.cuda.synchronize()
        t_rank = time.perf_counter() - t0            # this rank's own time, before the closing barrier
        if pg is not None:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    if pg is not None:
        torch.distributed.all_reduce(elapsed, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    loss = float(m["loss"].item())
    ks = timer.summary()
    dist = exchange_summary(trainer.exchange_events, trainer.exchange_log, args.steps, t_rank, pg, world, device)

    teacher_ms = None
    if not args.no_teacher_fwd:
        # teacher forward (large-v2 encoder + decoder over T_dec 447 + head) ms/clip
        wav, dec, lab = batches[0]
        mel, conv = fe.extract(wav)
        if args.dtype == "fp16":
            conv = teacher.conv_input(mel)
        for rep in range(4):
            if rep == 1:
                torch.cuda.synchronize()
                ta = time.perf_counter()
            enc = teacher.encode(conv)
            teacher.lm_head(teacher.decode(dec, enc, enc.shape[0] // args.batch))
        torch.cuda.synchronize()
        teacher_ms = (time.perf_counter() - ta) / 3 / args.batch * 1e3

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline()

    if rank == 0:
        value = args.steps * args.batch * world / elapsed
        flops_clip = _flops_per_clip(student.config, teacher.config, trainer.share)
        roof = None
        if ks is not None:
            achieved = ks["rate"] / 1e12
            c3b = args.config == "c3" and args.dtype == "bf16"      # the committed PMC summaries are of the bf16 c3 step
            pmc, pmc_src = load_pmc("gemm_nn") if c3b else (None, None)
            roof = dict(bound="mfma", achieved=round(achieved, 2), peak=PEAK_BF16_TFLOPS, unit="TFLOP/s",
                        frac=round(achieved / PEAK_BF16_TFLOPS, 4), traffic=pmc,
                        mfma_busy_frac=(load_mfma("c3_step", "gemm_pp (persistent 256x256 forward GEMM)")
                                        if c3b else None),
                        kernel=f"hand-written tw_gemm_{args.dtype} K-major x K-major launches (the forward X.W^T with fused "
                               "epilogues: GELU fc1, residual out_proj/fc2 of bf16 streams, long-K fc2): "
                               "gemm_pp_kernel (persistent 256x256 ping-pong, + split-K tail) + "
                               "gemm_kernel<false,false,128,...> for grids under ~1000 256-tiles",
                        launches_per_step=ks["launches"] // args.steps, avg_launch_ms=round(ks["avg_ms"], 4),
                        algo_tflop_per_launch=round(ks["avg_work"] / 1e12, 4),
                        algo_bytes_per_launch=round(ks["avg_bytes"]),
                        traffic_over_algo=(round(pmc / ks["avg_bytes"], 3) if pmc and ks["avg_bytes"] else None),
                        # read from committed files, not measured in this run (see each file's `source`)
                        traffic_source=pmc_src,
                        mfma_busy_source=_committed(MFMA_FILE)[1] if c3b else None)
        out = {
            "metric": "distillation utterances/sec (30 s clips)",
            "value": round(value, 3), "unit": "utt/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (30 s 16 kHz sines + noise, random-init weights, SURVEY.md §8d labels)",
            "config": {"workload": ("c3: distil-32-2 student <- whisper-large-v2 teacher, frozen shared encoder"
                                    if args.config == "c3" else
                                    "c2: whisper-small student <- whisper-large-v2 teacher, full teacher fwd"),
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch, "seq_len": 447,
                       "parallelism": f"dp{world}"},
            "teacher_fwd_ms_per_clip": None if teacher_ms is None else round(teacher_ms, 3),
            # north-star target (>= 40 % MFMA on the large-v2 teacher forward), two readings: the algorithmic
            # 3.445 TFLOP/clip over the measured time vs the 2.5 PF nominal peak, and the MFMA-busy counter
            # share of SIMD-cycles from the committed PMC pass (profiles/mfma_latest.json)
            "teacher_fwd_mfma_frac": None if teacher_ms is None else round(3.445 / teacher_ms / PEAK_BF16_TFLOPS * 1e3, 4),
            "teacher_fwd_mfma_busy_frac": load_mfma("teacher_forward", "ALL_BUT_OTHER"),
            "teacher_fwd_mfma_busy_source": _committed(MFMA_FILE)[1],
            "model_tflops_per_step_per_gpu": round(flops_clip * args.batch / 1e12, 2),
            "step_mfma_frac": round(flops_clip * value / world / 1e12 / PEAK_BF16_TFLOPS, 4),
            "final_loss": round(loss, 4),
            "roofline": roof,
            "distributed": dist,
            # fp16: accelerate's GradScaler state after the timed steps (a skipped step is timed like any other)
            "loss_scaler": (None if trainer.scaler is None else
                            {"scale": trainer.scaler.scale, "skipped_steps": trainer.skipped_steps}),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if pg is not None:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
