"""One attention-forward shape (default: the large-v2 encoder self-attention, B = 64, H = 20, T = 1500) run
`--reps` times, for rocprofv3 --pmc passes over the forward kernel alone."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from tw import ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tq", type=int, default=1500)
    ap.add_argument("--tk", type=int, default=1500)
    ap.add_argument("--causal", type=int, default=0)
    a = ap.parse_args()
    dev = "cuda"
    B, H = 64, 20
    d = H * 64
    q = torch.randn(B * a.tq, 3 * d, device=dev).bfloat16()
    kv = torch.randn(B * a.tk, 2 * d, device=dev).bfloat16()
    o = torch.empty(B * a.tq, d, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H * a.tq, device=dev)
    for _ in range(a.reps):
        ops.attn_fwd(q, 3 * d, kv, 2 * d, kv[:, d:], 2 * d, o, d, lse, B, H, a.tq, a.tk, a.causal, 0.125)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
