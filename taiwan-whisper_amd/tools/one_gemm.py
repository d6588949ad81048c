"""Run one GEMM shape a few times (for rocprofv3 counter collection).

    python tools/one_gemm.py M N K [flags]     (flags: ops.GEMM_TILE* forced-tile bits, default 0)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

M, N, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
force = int(sys.argv[4]) if len(sys.argv) > 4 else 0
A = torch.randn(M, K, device="cuda").bfloat16()
B = torch.randn(N, K, device="cuda").bfloat16()
C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
for _ in range(4):
    ops.gemm(A, B, C, M, N, K, lda=K, ldb=K, ldc=N, flags=ops.GEMM_ROUND | force)
torch.cuda.synchronize()
