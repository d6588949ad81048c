"""Run the encoder-shape attention forward a few times (for rocprofv3 counter collection).
Variant via TW_ATTN_FWD (0 = 16x16 kernel, 4 / 8 = 32x32 kernel with that many waves)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops

B, H, T = 64, 20, 1500
d = H * 64
q = torch.randn(B * T, 3 * d, device="cuda").bfloat16()
kv = torch.randn(B * T, 2 * d, device="cuda").bfloat16()
o = torch.empty(B * T, d, dtype=torch.bfloat16, device="cuda")
lse = torch.empty(B * H * T, device="cuda")
for _ in range(4):
    ops.attn_fwd(q, 3 * d, kv, 2 * d, kv[:, d:], 2 * d, o, d, lse, B, H, T, T, False, 0.125)
torch.cuda.synchronize()
