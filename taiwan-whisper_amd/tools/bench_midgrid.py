"""Tile A/B on mid-size forward grids (c2: teacher encoder at B = 32, M = 48000; the whisper-small student's
d = 768 shapes; teacher decoder at B = 32 / 64): 128x128 vs persistent 256x256 (pp) vs 256x256, plain
bf16 output with bias + round and with the in-place bf16 residual.  Interleaved rounds, one process."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

VARIANTS = (("t128", ops.GEMM_TILE128), ("pp", ops.GEMM_TILE256PP), ("t256", ops.GEMM_TILE256))
SHAPES = [(48000, 1280, 1280, True), (48000, 1280, 5120, True), (48000, 768, 768, True), (48000, 768, 3072, True),
          (48000, 2304, 768, False), (48000, 3072, 768, False), (14304, 1280, 1280, True), (14304, 1280, 5120, True),
          (14304, 768, 768, True), (28608, 1280, 1280, True), (28608, 1280, 5120, True), (64000, 1280, 1280, True)]


def main(rounds=5):
    for M, N, K, res in SHAPES:
        A = torch.randn(M, K, device="cuda").bfloat16()
        W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        C = torch.randn(M, N, device="cuda").bfloat16()

        def run(f):
            ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=b, res=C if res else None, ldr=N if res else 0,
                     flags=ops.GEMM_ROUND | f)
        for _, f in VARIANTS:
            run(f)
        times = {v: [] for v, _ in VARIANTS}
        for _ in range(rounds):
            for v, f in VARIANTS:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    run(f)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / 3)
        fl = 2.0 * M * N * K
        t256 = ((M + 255) // 256) * ((N + 255) // 256)
        line = f"M={M:6d} N={N:5d} K={K:5d} res={int(res)} tiles256={t256:5d} "
        for v, _ in VARIANTS:
            t = sorted(times[v])[rounds // 2]
            line += f" {v}: {t * 1e3:7.1f}us {fl / t / 1e9:6.0f}TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
