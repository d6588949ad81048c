"""Attention kernel timings on the step's shapes (encoder self 1500^2, decoder causal 447^2, cross 447x1500)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops


def main():
    dev = "cuda"
    torch.manual_seed(0)
    B, H = 64, 20
    d = H * 64
    for name, Tq, Tk, causal in (("enc self", 1500, 1500, False), ("dec self", 447, 447, True),
                                 ("cross", 447, 1500, False)):
        q = torch.randn(B * Tq, 3 * d, device=dev).bfloat16()
        kv = torch.randn(B * Tk, 2 * d, device=dev).bfloat16()
        o = torch.empty(B * Tq, d, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(B * H * Tq, device=dev)
        fn = lambda: ops.attn_fwd(q, 3 * d, kv, 2 * d, kv[:, d:], 2 * d, o, d, lse, B, H, Tq, Tk, causal, 0.125)
        for _ in range(2):
            fn()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 3)
        t = sorted(ts)[2]
        fl = 4.0 * B * H * Tq * Tk * 64 * (0.5 if causal else 1.0)
        csum = int(o.view(torch.int16).to(torch.int64).sum()) ^ int(lse.view(torch.int32).to(torch.int64).sum())
        print(f"fwd {name:9s} {t*1e3:8.1f}us {fl/t/1e9:7.1f} TF/s (causal counted at half)  bits {csum}", flush=True)
        do = torch.randn(B * Tq, d, device=dev).bfloat16()
        dq = torch.empty(B * Tq, d, dtype=torch.bfloat16, device=dev)
        dkv = torch.empty(B * Tk, 2 * d, dtype=torch.bfloat16, device=dev)
        fb = lambda: ops.attn_bwd(q, 3 * d, kv, 2 * d, kv[:, d:], 2 * d, o, d, do, d, lse, dq, d, dkv, 2 * d,
                                  dkv[:, d:], 2 * d, B, H, Tq, Tk, causal, 0.125)
        fb()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            fb()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 3
        print(f"bwd {name:9s} {t*1e3:8.1f}us {2.5*fl/t/1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
