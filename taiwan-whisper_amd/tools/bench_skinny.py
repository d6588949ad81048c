"""Decode-step GEMM shapes (M = batch rows): skinny weight-streaming kernel vs the forced 128x128
tile, interleaved rounds in one process; reports us and effective weight GB/s."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops


def t(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    for M in (64, 128):
        for N, K in ((1280, 1280), (3840, 1280), (5120, 1280), (1280, 5120), (51904, 1280)):
            A = torch.randn(M, K, device="cuda").bfloat16()
            W = torch.randn(N, K, device="cuda").bfloat16()
            C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            line = f"M={M:4d} N={N:6d} K={K:5d} "
            for nm, f in (("skinny", 0), ("t128", ops.GEMM_TILE128)):
                ms = t(lambda: ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, flags=ops.GEMM_ROUND | f))
                line += f"{nm}: {ms*1e3:7.1f}us {N*K*2/ms/1e6:7.1f}GB/s  "
            print(line, flush=True)


if __name__ == "__main__":
    main()
