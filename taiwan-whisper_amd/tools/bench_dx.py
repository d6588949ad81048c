"""Input-gradient GEMMs of the trainable student (dX = dY · W, W stored [N_out][K_in]) two ways, same box:
  nt : tw_gemm_bf16 with b_trans (W as stored: the 128² / 256² transposed-operand kernels);
  pp : W transposed once into a K-major copy (torch transpose + contiguous, timed) and the forward-GEMM route
       (persistent 256² kernel / whole-round + tail split).
Shapes: whisper-small student (c2, B = 32: M = 48 000 encoder rows, 14 304 decoder rows) and the distil-32-2
decoder (c3, M = 28 608)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

SHAPES = [("c2 enc qkv", 48000, 2304, 768), ("c2 enc out", 48000, 768, 768), ("c2 enc fc1", 48000, 3072, 768),
          ("c2 enc fc2", 48000, 768, 3072), ("c3 dec fc1", 28608, 5120, 1280), ("c3 dec out", 28608, 1280, 1280)]


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


def main():
    dev = "cuda"
    for name, M, N, K in SHAPES:          # dY [M][N], W [N][K] -> dX [M][K]
        g = torch.randn(M, N, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev).bfloat16()
        c1 = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
        c2 = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
        nt = lambda: ops.gemm(g, w, c1, M, K, N, lda=N, ldb=K, ldc=K, b_trans=True, flags=ops.GEMM_ROUND)

        def pp():
            wt = w.t().contiguous()
            ops.gemm(g, wt, c2, M, K, N, lda=N, ldb=N, ldc=K, flags=ops.GEMM_ROUND)
        nt()
        pp()
        torch.cuda.synchronize()
        same = torch.equal(c1, c2)
        tr = t(lambda: w.t().contiguous())
        a, b = t(nt), t(pp)
        fl = 2.0 * M * N * K
        print(f"{name:11s} M={M:6d} N={N:5d} K={K:5d} same={same}  nt {a*1e3:7.1f}us {fl/a/1e9:6.1f}TF  "
              f"pp+transpose {b*1e3:7.1f}us {fl/b/1e9:6.1f}TF  (transpose {tr*1e3:5.1f}us)", flush=True)


if __name__ == "__main__":
    main()
