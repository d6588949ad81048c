"""tw_decode_attn A/B on the decode shapes: cross-attention over 1500 encoder frames (large-v2: H = 20)
at batch 1 / 16 / 64 / 128 (bf16), or the batches and dtype given (`fp16 512`: the c4 pseudo-labelling shape);
`self` adds the graph-captured self-attention shape (Tk = 1 + *t_dev over a [B][448][2d] cache, t_dev = 200).
Prints us per call and the K/V read rate."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops


def main():
    H, Tk, d = 20, 1500, 1280
    dt = torch.float16 if "fp16" in sys.argv[1:] else torch.bfloat16
    batches = [int(a) for a in sys.argv[1:] if a.isdigit()] or [1, 16, 64, 128]
    for B in batches:
        kv = torch.randn(B * Tk, 2 * d, device="cuda").to(dt)
        q = torch.randn(B, d, device="cuda").to(dt)
        o = torch.empty(B, d, dtype=dt, device="cuda")
        run = lambda: ops.decode_attn(q, d, kv, 2 * d, Tk * 2 * d, kv[:, d:], 2 * d, Tk * 2 * d, o, d, B, H, Tk, 0.125)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        print(f"{str(dt)[6:]} B={B:4d}: {us:8.1f} us  {B * Tk * 2 * d * 2 / us / 1e3:7.1f} GB/s",
              flush=True)
        if "self" in sys.argv[1:]:
            T_max, t = 448, 200
            cache = torch.randn(B, T_max, 2 * d, device="cuda").to(dt)
            qkv = torch.randn(B, 3 * d, device="cuda").to(dt)
            t_dev = torch.full((1,), t, dtype=torch.int32, device="cuda")
            sb = T_max * 2 * d
            run = lambda: ops.decode_attn(qkv, 3 * d, cache, 2 * d, sb, cache.view(-1)[d:], 2 * d, sb, o, d, B, H, 1,
                                          0.125, tk_dev=t_dev, tk_max=T_max)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(50):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 50 * 1e3
            print(f"{str(dt)[6:]} self B={B:4d} Tk={t + 1}: {us:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
