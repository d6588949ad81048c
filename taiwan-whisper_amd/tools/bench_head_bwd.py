"""LM-head backward products at c3 (M = 64 x 447 rows, V = 51904 padded vocabulary, d = 1280): dX = dlogits . E
(E MN-major) and dW = dlogits^T . h, per forced tile variant (interleaved, one process, random data)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops


def timeit(fn, reps=3, rounds=5):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[len(ts) // 2]


def main():
    M, V, d = 28608, 51904, 1280
    dl = torch.randn(M, V, device="cuda").bfloat16()
    E = torch.randn(V, d, device="cuda").bfloat16()
    dx = torch.empty(M, d, device="cuda")
    fl = 2.0 * M * V * d
    for name, f in (("t128", ops.GEMM_TILE128), ("t256", ops.GEMM_TILE256), ("dflt", 0)):
        t = timeit(lambda: ops.gemm(dl, E, dx, M, d, V, lda=V, ldb=d, ldc=d, b_trans=True, flags=f))
        print(f"dX  {name:5s} {t*1e3:8.1f} us {fl/t/1e9:7.1f} TF/s", flush=True)
    Et = E.t().contiguous()      # K-major B: the persistent kernel's layout
    for name, f in (("pp", ops.GEMM_TILE256PP), ("dflt", 0)):
        t = timeit(lambda: ops.gemm(dl, Et, dx, M, d, V, lda=V, ldb=V, ldc=d, flags=f))
        print(f"dX K-major B {name:5s} {t*1e3:8.1f} us {fl/t/1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()


def vendor_nn():
    """the same dX products (B MN-major) on hipBLASLt through torch.matmul, and the student decoder's dX shapes"""
    for name, M, N, K in (("head dX", 28608, 1280, 51904), ("qkv dX", 28608, 1280, 3840),
                          ("fc2 dX", 28608, 5120, 1280), ("out dX", 28608, 1280, 1280)):
        g = torch.randn(M, K, device="cuda").bfloat16()
        W = torch.randn(K, N, device="cuda").bfloat16()
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        ours = timeit(lambda: ops.gemm(g, W, out, M, N, K, lda=K, ldb=N, ldc=N, b_trans=True, flags=ops.GEMM_ROUND))
        lt = timeit(lambda: torch.matmul(g, W, out=out))
        fl = 2.0 * M * N * K
        print(f"NN {name:8s} ours {ours*1e3:8.1f} us {fl/ours/1e9:7.1f} TF/s   hipBLASLt {lt*1e3:8.1f} us "
              f"{fl/lt/1e9:7.1f} TF/s", flush=True)
        del g, W, out


if __name__ == "__main__" and os.environ.get("VENDOR_NN"):
    vendor_nn()
