"""Forward-GEMM rate on selected step shapes under the current TW_GEMM_GROUP_M (read once per process:
run once per value).  usage: TW_GEMM_GROUP_M=g python bench_group.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops
from bench_vendor import timeit

SHAPES = [("lm head", 28608, 51904, 1280), ("dec qkv", 28608, 3840, 1280), ("dec fc1", 28608, 5120, 1280),
          ("xattn kv", 96000, 2560, 1280), ("enc fc1", 96000, 5120, 1280)]


def main():
    g = os.environ.get("TW_GEMM_GROUP_M", "default")
    for name, M, N, K in SHAPES:
        A = torch.randn(M, K, device="cuda").bfloat16()
        W = torch.randn(N, K, device="cuda").bfloat16()
        C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        t = timeit(lambda: ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, flags=ops.GEMM_ROUND))
        print(f"group {g:7s} {name:9s} {t*1e3:8.1f} us {2.0*M*N*K/t/1e9:7.1f} TF/s", flush=True)
        del A, W, C


if __name__ == "__main__":
    main()
