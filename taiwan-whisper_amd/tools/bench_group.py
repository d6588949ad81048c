"""Forward-GEMM time per tile order (group_m = runs of m-tiles walked n-tile by n-tile; 1 = row-major) on the step's
shapes, the variants interleaved in ONE process (flags bits 24-27 force group_m per call).
usage: python bench_group.py [g1,g2,...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

SHAPES = [("enc qkv", 96000, 3840, 1280), ("enc fc1", 96000, 5120, 1280), ("enc fc2", 96000, 1280, 5120),
          ("xattn kv", 96000, 2560, 1280), ("lm head", 28608, 51904, 1280), ("dec qkv", 28608, 3840, 1280),
          ("dec fc1", 28608, 5120, 1280)]


def main():
    groups = [int(g) for g in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,8").split(",")]
    for name, M, N, K in SHAPES:
        A = torch.randn(M, K, device="cuda").bfloat16()
        W = torch.randn(N, K, device="cuda").bfloat16()
        C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        run = lambda g: ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, flags=ops.GEMM_ROUND | (g << 24))
        for g in groups:
            run(g)
        ts = {g: [] for g in groups}
        for _ in range(5):
            for g in groups:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    run(g)
                e1.record()
                torch.cuda.synchronize()
                ts[g].append(e0.elapsed_time(e1) / 3)
        line = f"{name:9s} M={M:6d} N={N:6d} K={K:5d} "
        for g in groups:
            t = sorted(ts[g])[2]
            line += f" g{g}: {t*1e3:7.1f}us {2.0*M*N*K/t/1e9:6.0f}TF"
        print(line, flush=True)
        del A, W, C


if __name__ == "__main__":
    main()
