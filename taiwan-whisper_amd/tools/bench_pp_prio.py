"""A/B of the persistent ping-pong GEMM's issue-priority schemes (gemm_pp_kernel<PRIO>, flags bits 15-16)
and its epilogue cost (p4e: no epilogue, p4z: the epilogue computed and stored into tile 0 -- L2-resident
stores, no HBM write traffic; p4s: the epilogue computed, nothing stored -- needs tools/patches/pp_epilogue_nostore_diag.patch applied, and
that build perturbs the epilogue code (per-store branches); diagnostic flags),
interleaved in one process on random data, forward shapes of the distillation step."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

SHAPES = [("enc qkv", 96000, 3840, 1280, 0), ("enc out", 96000, 1280, 1280, 0), ("enc fc1", 96000, 5120, 1280, 1),
          ("enc fc2", 96000, 1280, 5120, 0), ("xattn kv", 96000, 2560, 1280, 0), ("dec fc1", 28608, 5120, 1280, 1),
          ("lm head", 28608, 51904, 1280, 0)]
VARIANTS = (sys.argv[1] if len(sys.argv) > 1 else "p4,p0,p4e").split(",")
DT = torch.float16 if "fp16" in sys.argv[2:] else torch.bfloat16     # `... p4 fp16`: the fp16 instantiation
FLAG = {"p4": 0, "p4e": 4096, "p4z": 1 << 20, "p4s": 1 << 21, "p0": 1 << 15, "p0e": (1 << 15) | 4096,
        "p2x": 2 << 15, "p2xe": (2 << 15) | 4096, "p1": 3 << 15, "p5e": (5 << 15) | 4096, "p6e": (6 << 15) | 4096, "p7e": (7 << 15) | 4096,
        "p4l": 1 << 22, "p4le": (1 << 22) | 4096}     # p4l*: diagnostic build, panels of one block per XCD (L2 hits)


def vflag(v):
    return ops.GEMM_TILE256PP | FLAG[v]


def main(rounds=5):
    dev = "cuda"
    for name, M, N, K, gelu in SHAPES:
        A = torch.randn(M, K, device=dev).to(DT)
        W = torch.randn(N, K, device=dev).to(DT)
        C = torch.empty(M, N, dtype=DT, device=dev)
        bias = torch.randn(N, device=dev).to(DT)
        base = ops.GEMM_ROUND

        def run(v):
            if gelu:
                ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bias, flags=base | ops.GEMM_GELU | vflag(v))
            else:
                ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bias, flags=base | vflag(v))
        outs = {}
        for v in VARIANTS:
            run(v)
            outs[v] = C.clone()
        same = all(torch.equal(outs[v], outs[VARIANTS[0]]) for v in VARIANTS if v in ('p0', 'p1', 'p4'))
        times = {v: [] for v in VARIANTS}
        for _ in range(rounds):
            for v in VARIANTS:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    run(v)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / 3)
        fl = 2.0 * M * N * K
        line = f"{name:9s} M={M:6d} N={N:6d} K={K:5d} same={same} "
        for v in VARIANTS:
            t = sorted(times[v])[rounds // 2]
            mult = 2 if v.startswith("p2x") else 1       # doubled MFMA phases: twice the matrix work
            line += f" {v}: {mult * fl / t / 1e9:7.1f}TF"
        print(line, flush=True)
        del A, W, C, outs


if __name__ == "__main__":
    main()
