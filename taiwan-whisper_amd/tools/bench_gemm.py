"""Interleaved A/B timing of the GEMM tile variants on the distillation step's shapes
(MI355X_MICROARCH/cdna_hip_programming §5.4 rule 24: variants x rounds in ONE process, random data)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

VARIANTS = (("dflt", 0), ("t128", 256), ("t256", 512), ("s3", 1024), ("pp", 2048))   # dflt: the library's own pick
SHAPES = [  # (name, M, N, K, a_trans, b_trans)
    ("enc qkv", 96000, 3840, 1280, 0, 0), ("enc out", 96000, 1280, 1280, 0, 0),
    ("enc fc1", 96000, 5120, 1280, 0, 0), ("enc fc2", 96000, 1280, 5120, 0, 0),
    ("xattn kv", 96000, 2560, 1280, 0, 0), ("dec fc1", 28608, 5120, 1280, 0, 0),
    ("dec out", 28608, 1280, 1280, 0, 0), ("lm head", 28608, 51904, 1280, 0, 0),
    ("dec qkv", 28608, 3840, 1280, 0, 0), ("dec fc2", 28608, 1280, 5120, 0, 0),
    ("dW fc1", 5120, 1280, 28608, 1, 1), ("dX fc2", 28608, 5120, 1280, 0, 1),
    ("dW head", 51904, 1280, 28608, 1, 1), ("dX head", 28608, 1280, 51904, 0, 1),
]


# config 2 (whisper-small student d = 768 at B = 32: encoder rows 48 000, decoder rows 14 304; trainable encoder):
# forward and the backward dX (W transposed) / dW (both transposed, K = tokens) products
SHAPES_C2 = [
    ("s enc qkv", 48000, 2304, 768, 0, 0), ("s enc out", 48000, 768, 768, 0, 0), ("s enc fc1", 48000, 3072, 768, 0, 0),
    ("s enc fc2", 48000, 768, 3072, 0, 0), ("s dec qkv", 14304, 2304, 768, 0, 0), ("s lm head", 14304, 51904, 768, 0, 0),
    ("s dX fc1", 48000, 768, 3072, 0, 1), ("s dX fc2", 48000, 3072, 768, 0, 1), ("s dX qkv", 48000, 768, 2304, 0, 1),
    ("s dW fc1", 3072, 768, 48000, 1, 1), ("s dW fc2", 768, 3072, 48000, 1, 1), ("s dW qkv", 2304, 768, 48000, 1, 1),
    ("s dW out", 768, 768, 48000, 1, 1), ("s dX head", 14304, 768, 51904, 0, 1), ("s dW head", 51904, 768, 14304, 1, 1),
    ("s dec out", 14304, 768, 768, 0, 0), ("s dec fc2", 14304, 768, 3072, 0, 0), ("s dec fc1", 14304, 3072, 768, 0, 0),
    ("s dX decfc1", 14304, 768, 3072, 0, 1), ("s xkv", 48000, 1536, 768, 0, 0),
    ("t enc out", 48000, 1280, 1280, 0, 0), ("t enc fc1", 48000, 5120, 1280, 0, 0), ("t dec out", 14304, 1280, 1280, 0, 0),
]


def main(rounds=5, only=None):
    dev = "cuda"
    res = {}
    shapes = SHAPES_C2 if only == ["c2"] else SHAPES
    for name, M, N, K, at, bt in shapes:
        if only and only != ["c2"] and not any(o in name for o in only):
            continue
        A = (torch.randn(K, M, device=dev) if at else torch.randn(M, K, device=dev)).to(torch.bfloat16)
        B = (torch.randn(K, N, device=dev) if bt else torch.randn(N, K, device=dev)).to(torch.bfloat16)
        C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        for variant, flag in VARIANTS:
            for _ in range(2):
                ops.gemm(A, B, C, M, N, K, lda=M if at else K, ldb=N if bt else K, ldc=N, a_trans=bool(at),
                         b_trans=bool(bt), flags=ops.GEMM_ROUND | flag)
        times = {v: [] for v, _ in VARIANTS}
        for r in range(rounds):
            for variant, flag in VARIANTS:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    ops.gemm(A, B, C, M, N, K, lda=M if at else K, ldb=N if bt else K, ldc=N, a_trans=bool(at),
                             b_trans=bool(bt), flags=ops.GEMM_ROUND | flag)
                e1.record()
                torch.cuda.synchronize()
                times[variant].append(e0.elapsed_time(e1) / 3)
        fl = 2.0 * M * N * K
        line = f"{name:10s} M={M:6d} N={N:6d} K={K:6d} "
        for v, _ in VARIANTS:
            t = sorted(times[v])[len(times[v]) // 2]
            line += f"{v}: {t*1e3:8.1f}us {fl/t/1e9:7.1f}TF  "
        print(line, flush=True)


if __name__ == "__main__":
    main(only=sys.argv[1].split(",") if len(sys.argv) > 1 else None)
