"""Ping-pong GEMM diagnostics: persistent vs one-tile-per-block, with / without the epilogue
(debug flag bits 4096 = skip epilogue, 8192 = one tile per workgroup); interleaved rounds."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

VARIANTS = (("pp", 0), ("noepi", 4096))


def main(rounds=5):
    for M, N, K in ((96000, 5120, 1280), (28608, 3840, 1280), (28608, 51904, 1280), (96000, 1280, 5120)):
        A = torch.randn(M, K, device="cuda").bfloat16()
        B = torch.randn(N, K, device="cuda").bfloat16()
        C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        bias = torch.randn(N, device="cuda").bfloat16()
        run = lambda f: ops.gemm(A, B, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bias, flags=ops.GEMM_ROUND | ops.GEMM_BIAS | ops.GEMM_TILE256PP | f)
        for _, f in VARIANTS:
            run(f); run(f)
        t = {v: [] for v, _ in VARIANTS}
        for _ in range(rounds):
            for v, f in VARIANTS:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    run(f)
                e1.record()
                torch.cuda.synchronize()
                t[v].append(e0.elapsed_time(e1) / 3)
        fl = 2.0 * M * N * K
        line = f"M={M:6d} N={N:5d} K={K:5d}\n"
        for v, _ in VARIANTS:
            ms = sorted(t[v])[len(t[v]) // 2]
            line += f"   {v:14s}: {ms*1e3:7.1f}us {fl/ms/1e9:6.1f}TF\n"
        print(line, flush=True)


if __name__ == "__main__":
    main()
