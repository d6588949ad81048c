"""The persistent forward GEMM (gemm_pp_kernel, forced with GEMM_TILE256PP) on the step's K-major shapes with their
epilogues (bias + round, GELU, bf16 residual): median time and TF/s per shape, and a checksum of each output so that two
libraries run alternately (tools/calls/ab.sh, TW_HIP_LIB) can be checked for identical bits.  Round 5 used it first
for the 4-slot ring kernel against the two-buffer one (PP2 = flag 1 << 21 in that build,
tools/patches/gemm_ring_32k_4slot.patch; profiles/r05_b_*).

    python tools/bench_ring.py [rounds] [extra flags]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

VARIANTS = [("tree", 0)]
SHAPES = [  # (name, M, N, K, epilogue)
    ("enc qkv", 96000, 3840, 1280, "bias"), ("enc out", 96000, 1280, 1280, "res"),
    ("enc fc1", 96000, 5120, 1280, "gelu"), ("enc fc2", 96000, 1280, 5120, "res"),
    ("xattn kv", 96000, 2560, 1280, "bias"), ("dec fc1", 28608, 5120, 1280, "gelu"),
    ("dec qkv", 28608, 3840, 1280, "bias"), ("lm head", 28608, 51904, 1280, "plain"),
]


def main(rounds=5):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    tot = {v: 0.0 for v, _ in VARIANTS}
    for name, M, N, K, epi in SHAPES:
        A = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        B = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        bias = torch.randn(N, device=dev, generator=g).to(torch.bfloat16)
        res = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16) if epi == "res" else None
        f = ops.GEMM_ROUND | ops.GEMM_TILE256PP
        kw = {}
        if epi != "plain":
            f |= ops.GEMM_BIAS
            kw["bias"] = bias
        if epi == "gelu":
            f |= ops.GEMM_GELU
        if epi == "res":
            f |= ops.GEMM_RES
            kw.update(res=res, ldr=N)
        outs = {}
        for v, extra in VARIANTS:
            C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            ops.gemm(A, B, C, M, N, K, lda=K, ldb=K, ldc=N, flags=f | extra, **kw)
            outs[v] = C
        torch.cuda.synchronize()
        same = all(torch.equal(outs[v], outs[VARIANTS[0][0]]) for v, _ in VARIANTS)
        csum = int(outs[VARIANTS[0][0]].view(torch.int16).to(torch.int64).sum())
        times = {v: [] for v, _ in VARIANTS}
        C = outs[VARIANTS[0][0]]
        for _ in range(rounds):
            for v, extra in VARIANTS:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    ops.gemm(A, B, C, M, N, K, lda=K, ldb=K, ldc=N, flags=f | extra, **kw)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / 3)
        fl = 2.0 * M * N * K
        line = f"{name:9s} M={M:6d} N={N:6d} K={K:5d} {epi:5s} identical={same} sum={csum} "
        for v, _ in VARIANTS:
            t = sorted(times[v])[len(times[v]) // 2]
            tot[v] += t
            line += f"{v}: {t*1e3:8.1f}us {fl/t/1e9:7.1f}TF  "
        print(line, flush=True)
        del A, B, C, outs, res
        torch.cuda.empty_cache()
    print("total " + "  ".join(f"{v} {tot[v]:.3f} ms" for v, _ in VARIANTS), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2:
        VARIANTS.append(("flag", int(sys.argv[2])))
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
