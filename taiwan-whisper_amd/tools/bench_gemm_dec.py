import os, sys
sys.path.insert(0, "taiwan-whisper_amd")
import torch
from tw import ops
V = (("t128", 256), ("s2", 262144), ("pp", 2048), ("dflt", 0))
for name, M, N, K, flags in (("dec out", 28608, 1280, 1280, 0), ("dec fc2", 28608, 1280, 5120, 0),
                             ("dec out res", 28608, 1280, 1280, 1), ("dec fc2 res", 28608, 1280, 5120, 1),
                             ("dec q", 28608, 1280, 1280, 2), ("enc out res", 96000, 1280, 1280, 1),
                             ("conv1", 192000, 1280, 240, 3)):
    A = torch.randn(M, K, device="cuda").bfloat16(); W = torch.randn(N, K, device="cuda").bfloat16()
    C = torch.randn(M, N, device="cuda").bfloat16(); bias = torch.randn(N, device="cuda").bfloat16()
    def run(f):
        if flags == 1:
            ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bias, res=C, ldr=N, flags=ops.GEMM_ROUND | f)
        else:
            ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bias, flags=ops.GEMM_ROUND | f)
    res = {}
    for v, f in V:
        for _ in range(2): run(f)
    ts = {v: [] for v, _ in V}
    for r in range(5):
        for v, f in V:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3): run(f)
            e1.record(); torch.cuda.synchronize(); ts[v].append(e0.elapsed_time(e1) / 3)
    fl = 2.0 * M * N * K
    print(f"{name:12s} " + "  ".join(f"{v}: {sorted(ts[v])[2]*1e3:7.1f}us {fl/sorted(ts[v])[2]/1e9:6.0f}TF" for v, _ in V), flush=True)
