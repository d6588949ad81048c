"""GELU epilogue sweep over every finite bf16 pre-activation: C = bf16(x) through each GEMM tile
variant's GELU epilogue vs the exact erf GELU rounded to bf16 (fp64 reference)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

bits = torch.arange(0, 65536, dtype=torch.int32).to(torch.int16)
x = bits.view(torch.bfloat16)
x = x[torch.isfinite(x.float())]
M = x.numel() // 256 * 256
x = x[:M]
K, N = 64, 256
A = torch.zeros(M, K, dtype=torch.bfloat16)
A[:, 0] = x
W = torch.zeros(N, K, dtype=torch.bfloat16)
W[:, 0] = 1.0
ref = (0.5 * x.double() * (1 + torch.erf(x.double() / 2 ** 0.5))).to(torch.bfloat16).float()
Ad, Wd = A.cuda(), W.cuda()
for name, f in (("t128", ops.GEMM_TILE128), ("t256", ops.GEMM_TILE256), ("pp", ops.GEMM_TILE256PP)):
    C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    ops.gemm(Ad, Wd, C, M, N, K, lda=K, ldb=K, ldc=N, flags=ops.GEMM_ROUND | ops.GEMM_GELU | f)
    torch.cuda.synchronize()
    got = C.float().cpu()
    col = got[:, 0]
    same_cols = bool((got == col[:, None]).all())
    d = (col - ref).abs()
    ulp = torch.where(ref != 0, ref.abs() * 2 ** -7, torch.full_like(ref, 1e-30))
    bad = d > ulp
    print(name, "same_cols", same_cols, "max abs diff", float(d.max()), "beyond 1 ulp", int(bad.sum()))
    if bad.any():
        for j in bad.nonzero()[:10, 0].tolist():
            print("   x", float(x[j]), "got", float(col[j]), "ref", float(ref[j]))
