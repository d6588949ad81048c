"""Config c4 throughput: large-v2 batched greedy decode, random-init bf16 weights,
synthetic 30 s features; eos is suppressed so every clip runs exactly --new-tokens steps
(deterministic work, as §8d prescribes: max_new_tokens 224).

    python tools/bench_decode.py [--batch 64] [--new-tokens 224] [--clips 128] [--eager]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--new-tokens", type=int, default=224)
    ap.add_argument("--clips", type=int, default=128)
    ap.add_argument("--config", default="large-v2")
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--longform-seconds", type=float, default=0.0,
                    help="config c5: one input of this many seconds, return_timestamps, --new-tokens per window")
    a = ap.parse_args()
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
    from oracle.weights import CONFIGS
    from tw.config import GenerationConfig, WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration, random_init_
    cfg = WhisperConfig(**CONFIGS[a.config])
    m = WhisperForConditionalGeneration(cfg, dtype=torch.bfloat16)
    random_init_(m, seed=0)
    m.generation_config = GenerationConfig(suppress_tokens=[50257], begin_suppress_tokens=[220, 50257],
                                           lang_to_id={"<|zh|>": 50260})
    if a.longform_seconds > 0:
        T = int(a.longform_seconds * 100)
        lf = torch.randn(1, 80, T, device="cuda") * 0.3
        trace = []
        m.generate(lf[:, :, :3500], return_timestamps=True, language="zh", task="transcribe", max_new_tokens=8,
                   use_graph=not a.eager)                                                     # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = m.generate(lf, return_timestamps=True, language="zh", task="transcribe", max_new_tokens=a.new_tokens,
                         use_graph=not a.eager, _trace=trace)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        steps = sum(len(t["raw"]) for t in trace)
        print(f"c5 long-form {a.config}: {a.longform_seconds:.0f} s audio, {len(trace)} windows, {steps} decode steps, "
              f"{out.shape[1]} output tokens: {dt:.2f} s wall ({a.longform_seconds / dt:.1f}x real time, "
              f"{dt / max(steps, 1) * 1e3:.2f} ms/step at batch 1)", flush=True)
        return
    feats = torch.randn(a.batch, 80, 3000, device="cuda") * 0.3
    m.generate(feats[:2], language="zh", task="transcribe", max_new_tokens=4, use_graph=not a.eager)   # warm-up
    torch.cuda.synchronize()
    n_sub = max(1, a.clips // a.batch)
    t0 = time.perf_counter()
    for _ in range(n_sub):
        out = m.generate(feats, language="zh", task="transcribe", max_new_tokens=a.new_tokens,
                         use_graph=not a.eager)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    clips = n_sub * a.batch
    print(f"c4 greedy {a.config}: {clips} clips x {out.shape[1]} tokens, batch {a.batch}: {dt:.2f} s "
          f"-> {clips / dt:.2f} clips/s, {dt / n_sub / a.new_tokens * 1e3:.2f} ms/step "
          f"({'eager' if a.eager else 'graph'})", flush=True)


if __name__ == "__main__":
    main()
