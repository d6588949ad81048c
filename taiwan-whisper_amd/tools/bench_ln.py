"""LayerNorm kernel micro-bench: bf16/fp16 rows (the teacher / fp16 residual stream), plain and add+LN.
Prints achieved GB/s (algorithmic bytes: read x [+r], write y [+x_out], 2 B each) and max error vs torch."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from tw import ops  # noqa: E402


def run(rows, D, dt, add, reps=50):
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(rows, D, generator=g).to(dev, dt)
    r = torch.randn(rows, D, generator=g).to(dev, dt)
    w = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    b = (0.1 * torch.randn(D, generator=g)).to(dev)
    y = torch.empty_like(x)
    xo = torch.empty_like(x)

    def call():
        if add:
            ops.add_layernorm_fwd(x, r, xo, w, b, y)
        else:
            ops.layernorm_fwd(x, w, b, y)

    for _ in range(3):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    nbytes = rows * D * 2 * (4 if add else 2)
    xin = (x.float() + r.float()).to(dt) if add else x
    ref = torch.nn.functional.layer_norm(xin.float(), (D,), w, b, 1e-5).to(dt)
    err = (y.float() - ref.float()).abs().max().item()
    xerr = (xo.float() - xin.float()).abs().max().item() if add else 0.0
    print(f"rows={rows:6d} D={D} {str(dt):15s} add={int(add)} {us:8.1f} us {nbytes / us / 1e3:7.1f} GB/s "
          f"err={err:.3g} xerr={xerr:.3g}", flush=True)


if __name__ == "__main__":
    for dt in (torch.bfloat16, torch.float16):
        for rows in (448 * 64, 1500 * 64, 512):
            for add in ((False, True) if dt == torch.bfloat16 else (False,)):
                run(rows, 1280, dt, add)
