"""Cross-attention decode read rate by cache layout: the row-interleaved cross K/V the KV projection writes
([B*Tk][2d], head h at columns 64h.., key rows 2d*2 B apart) against a head-major copy ([B][H][Tk][64]:
one (clip, head) reads two contiguous 192 KB runs), emulated with the same kernel as B*H one-head clips.
Measurement only."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops
from bench_vendor import timeit


def main():
    H, Tk, d = 20, 1500, 1280
    for B in (64, 128, 512):
        kv = torch.randn(B * Tk, 2 * d, device="cuda").bfloat16()
        q = torch.randn(B, d, device="cuda").bfloat16()
        o = torch.empty(B, d, dtype=torch.bfloat16, device="cuda")
        t_row = timeit(lambda: ops.decode_attn(q, d, kv, 2 * d, Tk * 2 * d, kv[:, d:], 2 * d, Tk * 2 * d, o, d, B, H,
                                               Tk, 0.125), reps=10)
        kh = kv[:, :d].reshape(B, Tk, H, 64).transpose(1, 2).contiguous()      # [B][H][Tk][64]
        vh = kv[:, d:].reshape(B, Tk, H, 64).transpose(1, 2).contiguous()
        del kv
        oh = torch.empty(B * H, 64, dtype=torch.bfloat16, device="cuda")
        qh = q.reshape(B * H, 64).contiguous()
        t_hm = timeit(lambda: ops.decode_attn(qh, 64, kh, 64, Tk * 64, vh, 64, Tk * 64, oh, 64, B * H, 1, Tk, 0.125),
                      reps=10)
        same = torch.equal(oh.reshape(B, d), o)
        gb = B * Tk * 2 * d * 2 / 1e9
        print(f"B={B:4d}: row-interleaved {t_row*1e3:8.1f} us ({gb/t_row:6.2f} TB/s)  head-major {t_hm*1e3:8.1f} us "
              f"({gb/t_hm:6.2f} TB/s)  identical={same}", flush=True)
        del kh, vh


if __name__ == "__main__":
    main()
