"""Cost of the fused GEMM epilogues on the step's big shapes (interleaved rounds, one process)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops


def t(fn, rounds=5, reps=3):
    for _ in range(2):
        fn()
    out = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    return sorted(out)[len(out) // 2]


VARIANTS = (("t256", ops.GEMM_TILE256), ("s3", ops.GEMM_TILE256x128), ("pp", ops.GEMM_TILE256PP))
if os.environ.get("PP_ONLY"):
    VARIANTS = (("pp", ops.GEMM_TILE256PP),)


def main():
    dev = "cuda"
    M, K = 96000, 1280
    x = torch.randn(M, K, device=dev).bfloat16()
    for N, Kk, name in ((5120, 1280, "fc1"), (1280, 1280, "out"), (1280, 5120, "fc2")):
        A = torch.randn(M, Kk, device=dev).bfloat16()
        W = torch.randn(N, Kk, device=dev).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        Cf = torch.empty(M, N, dtype=torch.float32, device=dev)
        res = torch.randn(M, N, device=dev)
        resb = torch.randn(M, N, device=dev).bfloat16()
        fl = 2.0 * M * N * Kk
        cases = {
            "round bf16": lambda f: ops.gemm(A, W, Cb, M, N, Kk, lda=Kk, ldb=Kk, ldc=N, flags=ops.GEMM_ROUND | f),
            "bias+round": lambda f: ops.gemm(A, W, Cb, M, N, Kk, lda=Kk, ldb=Kk, ldc=N, bias=b,
                                             flags=ops.GEMM_ROUND | f),
            "bias+gelu": lambda f: ops.gemm(A, W, Cb, M, N, Kk, lda=Kk, ldb=Kk, ldc=N, bias=b,
                                            flags=ops.GEMM_ROUND | ops.GEMM_GELU | f),
            "f32 out": lambda f: ops.gemm(A, W, Cf, M, N, Kk, lda=Kk, ldb=Kk, ldc=N, flags=f),
            "bias+res f32 inplace": lambda f: ops.gemm(A, W, res, M, N, Kk, lda=Kk, ldb=Kk, ldc=N, bias=b, res=res,
                                                       ldr=N, flags=ops.GEMM_ROUND | f),
            "bias+res bf16 inplace": lambda f: ops.gemm(A, W, resb, M, N, Kk, lda=Kk, ldb=Kk, ldc=N, bias=b,
                                                        res=resb, ldr=N, flags=ops.GEMM_ROUND | f),
        }
        for cname, fn in cases.items():
            line = f"{name:4s} N={N:5d} K={Kk:5d} {cname:22s}"
            for vname, vf in VARIANTS:
                ms = t(lambda: fn(vf))
                line += f" {vname}: {ms*1e3:7.1f}us {fl/ms/1e9:6.1f}TF"
            print(line, flush=True)


if __name__ == "__main__":
    main()
