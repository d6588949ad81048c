"""Tile-variant A/B on the step's small-grid forward GEMMs (M = 64 x 447 decoder tokens, N = 1280:
< 1000 256-tiles, where the heuristic picks 128x128) with the epilogues they run in the step: bias
+ round (cross-attention q), bias + round + in-place bf16 residual (out_proj, fc2 of the teacher's
bf16 stream).  Interleaved rounds in one process, random data."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

VARIANTS = (("t128", ops.GEMM_TILE128), ("t256", ops.GEMM_TILE256), ("s3", ops.GEMM_TILE256x128),
            ("pp", ops.GEMM_TILE256PP))
SHAPES = [("q (bias)", 28608, 1280, 1280, False), ("out (res)", 28608, 1280, 1280, True),
          ("fc2 (res)", 28608, 1280, 5120, True)]


def main(rounds=7):
    for name, M, N, K, res in SHAPES:
        A = torch.randn(M, K, device="cuda").bfloat16()
        W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        C = torch.randn(M, N, device="cuda").bfloat16()

        def run(f):
            if res:
                ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=b, res=C, ldr=N, flags=ops.GEMM_ROUND | f)
            else:
                ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=b, flags=ops.GEMM_ROUND | f)
        for _, f in VARIANTS:
            run(f)
        times = {v: [] for v, _ in VARIANTS}
        for _ in range(rounds):
            for v, f in VARIANTS:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run(f)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / 5)
        fl = 2.0 * M * N * K
        line = f"{name:10s} M={M} N={N} K={K} "
        for v, _ in VARIANTS:
            t = sorted(times[v])[rounds // 2]
            line += f" {v}: {t * 1e3:7.1f}us {fl / t / 1e9:6.0f}TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
