"""Headroom check: our kernels vs the vendor libraries torch dispatches to on ROCm (hipBLASLt for
matmul, the SDPA flash backend for attention) on the distillation step's shapes, interleaved in one
process on random data.  Measurement only: nothing in the product calls the vendor path."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import torch.nn.functional as F

from tw import ops

GEMMS = [("enc qkv", 96000, 3840, 1280), ("enc out", 96000, 1280, 1280), ("enc fc1", 96000, 5120, 1280),
         ("enc fc2", 96000, 1280, 5120), ("xattn kv", 96000, 2560, 1280), ("dec qkv", 28608, 3840, 1280),
         ("dec out", 28608, 1280, 1280), ("dec fc1", 28608, 5120, 1280), ("dec fc2", 28608, 1280, 5120),
         ("lm head", 28608, 51904, 1280)]


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
    dev = "cuda"
    for name, M, N, K in GEMMS:
        A = torch.randn(M, K, device=dev).bfloat16()
        W = torch.randn(N, K, device=dev).bfloat16()
        C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        ours = timeit(lambda: ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, flags=ops.GEMM_ROUND))
        lt = timeit(lambda: torch.matmul(A, W.t(), out=C))
        fl = 2.0 * M * N * K
        print(f"gemm {name:9s} M={M:6d} N={N:6d} K={K:5d}  ours {fl/ours/1e9:7.1f} TF/s  hipBLASLt {fl/lt/1e9:7.1f} TF/s",
              flush=True)
        del A, W, C
    B, H = 64, 20
    d = H * 64
    for name, Tq, Tk, causal in (("enc self", 1500, 1500, False), ("dec self", 447, 447, True),
                                 ("cross", 447, 1500, False)):
        q = torch.randn(B * Tq, 3 * d, device=dev).bfloat16()
        kv = torch.randn(B * Tk, 2 * d, device=dev).bfloat16()
        o = torch.empty(B * Tq, d, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(B * H * Tq, device=dev)
        ours = timeit(lambda: ops.attn_fwd(q, 3 * d, kv, 2 * d, kv[:, d:], 2 * d, o, d, lse, B, H, Tq, Tk, causal,
                                           0.125))
        qt = q[:, :d].reshape(B, Tq, H, 64).transpose(1, 2).contiguous()
        kt = kv[:, :d].reshape(B, Tk, H, 64).transpose(1, 2).contiguous()
        vt = kv[:, d:].reshape(B, Tk, H, 64).transpose(1, 2).contiguous()
        try:
            from torch.nn.attention import SDPBackend, sdpa_kernel
            with sdpa_kernel([SDPBackend.FLASH_ATTENTION]):
                sd = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal))
        except Exception as e:  # backend unavailable on this build
            print(f"  sdpa flash unavailable: {type(e).__name__}: {e}")
            sd = float("nan")
        fl = 4.0 * B * H * Tq * Tk * 64 * (0.5 if causal else 1.0)
        print(f"attn {name:9s} ours {fl/ours/1e9:7.1f} TF/s  sdpa-flash {fl/sd/1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
