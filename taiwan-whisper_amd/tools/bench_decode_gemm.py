"""Decode-step Linears at batch M (c4: M = 128): the current route of tw_gemm_bf16 (skinny weight-streaming
kernel + split-K reduce, or 128x128 tiles) against hipBLASLt (torch.addmm: bias epilogue, bf16 out) on the
large-v2 decoder shapes.  Measurement only."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops
from bench_vendor import timeit

SHAPES = [("qkv", 3840, 1280), ("out/xq", 1280, 1280), ("fc1", 5120, 1280), ("fc2", 1280, 5120),
          ("lm head", 51904, 1280)]


def main():
    for M in (512, 256, 128):
        for name, N, K in SHAPES:
            A = torch.randn(M, K, device="cuda").bfloat16()
            W = torch.randn(N, K, device="cuda").bfloat16()
            b = torch.randn(N, device="cuda").bfloat16()
            C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            X = torch.randn(M, N, device="cuda").bfloat16()
            ours = timeit(lambda: ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=b, flags=ops.GEMM_ROUND),
                          reps=20)
            ours_res = timeit(lambda: ops.gemm(A, W, X, M, N, K, lda=K, ldb=K, ldc=N, bias=b, res=X, ldr=N,
                                               flags=ops.GEMM_ROUND), reps=20)
            lt = timeit(lambda: torch.addmm(b, A, W.t(), out=C), reps=20)
            mb = N * K * 2 / 1e6
            print(f"M={M:4d} {name:8s} N={N:6d} K={K:5d} ({mb:6.1f} MB W)  ours {ours*1e3:7.1f} us  ours+res "
                  f"{ours_res*1e3:7.1f} us  hipBLASLt {lt*1e3:7.1f} us ({mb/lt/1e3:6.2f} TB/s)", flush=True)
            del A, W, b, C, X


if __name__ == "__main__":
    main()
