"""The large-v2 decode step (config c5's unit of work) in isolation: ms per graph-replayed DecodeSession step at
batch 1 and at the fallback batch, the per-launch floor of a graph of dependent tiny launches, and each decode-step
Linear shape as a graph-captured chain of GEMV launches (us per launch).  With TW_HIP_LIB two libraries are compared
on one box (tools/calls/ab.sh); each line carries a checksum of the step's logits so that identical bits can be
checked.

    python tools/bench_step.py [reps] [batches, e.g. 1,6] [--step-only] [--copies] [--rows=N]

--copies: the batch's rows get B copies of the one window's encoder rows (a B-clip cross-K/V block, as before the
shared fallback-batch K/V) instead of the shared Tk rows.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch

from tw import ops as F


def _chain(fn, n=64, reps=10):
    """us per call of fn, from a graph holding n calls replayed reps times (median of 3 timings)."""
    g = torch.cuda.CUDAGraph()
    fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / (reps * n))
    return sorted(ts)[1]


def main(reps=20, batches=(1, 6), step_only=False, copies=False, rows=1):
    dev = "cuda"
    torch.manual_seed(0)
    t = torch.zeros(1, dtype=torch.int32, device=dev)
    if not step_only:
        _chains(t, rows)
    _steps(reps, batches, copies)


def _chains(t, rows=1):
    dev = "cuda"
    print(f"floor  step_advance chain {_chain(lambda: F.step_advance(t)):7.2f} us/launch", flush=True)
    h = torch.float16
    d, ffn = 1280, 5120
    x = (torch.randn(rows, d, device=dev) * 0.5).to(h)
    xf = (torch.randn(rows, ffn, device=dev) * 0.5).to(h)
    lnw, lnb = torch.rand(d, device=dev) + 0.5, torch.randn(d, device=dev) * 0.1
    for name, N, K, ln, res, fl in (("d x d  (out_proj, +res)", d, d, False, True, F.GEMM_ROUND),
                                    ("d x d  (LN + cross q)", d, d, True, False, F.GEMM_ROUND),
                                    ("3d x d (LN + qkv)", 3 * d, d, True, False, F.GEMM_ROUND),
                                    ("4d x d (LN + fc1 GELU)", ffn, d, True, False, F.GEMM_ROUND | F.GEMM_GELU),
                                    ("d x 4d (fc2, +res)", d, ffn, False, True, F.GEMM_ROUND)):
        W = (torch.randn(N, K, device=dev) * 0.02).to(h)
        b = (torch.randn(N, device=dev) * 0.1).to(h)
        C = torch.empty(rows, N, dtype=h, device=dev)
        r = torch.randn(rows, N, device=dev).to(h) if res else None
        a = xf if K == ffn else x
        kw = dict(bias=b, res=r, flags=fl)
        if ln:
            kw.update(ln_w=lnw, ln_b=lnb)
        us = _chain(lambda: F.gemv(a, W, C, **kw))
        print(f"gemv   {name:24s} x{rows} {us:7.2f} us/launch  {N * K * 2 / us / 1e3:7.1f} GB/s  "
              f"bits {int(C.view(torch.int16).to(torch.int64).sum())}", flush=True)


def _steps(reps, batches, copies=False):
    from oracle.weights import CONFIGS
    from tw.config import WhisperConfig
    from tw.generation import DecodeSession
    from tw.modeling import WhisperForConditionalGeneration, random_init_
    dev, h, d = "cuda", torch.float16, 1280
    cfg = WhisperConfig(**CONFIGS["large-v2"])
    m = random_init_(WhisperForConditionalGeneration(cfg, dtype=h, device=dev), seed=0)
    Tk = cfg.max_source_positions
    for B in batches:
        enc = (torch.randn(Tk, d, device=dev) * 0.5).to(h)
        sess = DecodeSession(m, enc.repeat(B, 1) if copies and B > 1 else enc, B, Tk, 256)
        sess.t_dev.fill_(100)
        sess.cur.fill_(50364)
        g = torch.cuda.CUDAGraph()
        sess.step()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            sess.step()
            F.step_advance(sess.t_dev, -1)      # every replay decodes position 100 again
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / reps)
        print(f"step   large-v2 fp16 batch {B}{' (K/V copies)' if copies and B > 1 else ''} at t=100  {sorted(ts)[1]:7.3f} ms/step  "
              f"bits {int(sess.logits.view(torch.int16).to(torch.int64).sum())}", flush=True)
        del sess, g


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(int(args[0]) if args else 20, tuple(int(b) for b in args[1].split(",")) if len(args) > 1 else (1, 6),
         "--step-only" in sys.argv, "--copies" in sys.argv,
         int(next((a.split("=")[1] for a in sys.argv if a.startswith("--rows=")), 1)))
