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


def run_bwd(rows, D, xdt, reps=30):
    """tw_layernorm_bwd with dx accumulated (the student's fp32 stream): algorithmic bytes = read x, dy, dx and
    write dx (the per-block dw / db partials and their reduction counted apart)."""
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(rows, D, generator=g).to(dev, xdt)
    dy = torch.randn(rows, D, generator=g).to(dev)
    w = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    mean = x.float().mean(1)
    rstd = (x.float().var(1, unbiased=False) + 1e-5).rsqrt()
    dx = torch.zeros(rows, D, device=dev)
    dw = torch.zeros(D, device=dev)
    db = torch.zeros(D, device=dev)
    call = lambda: ops.layernorm_bwd(x, w, mean, rstd, dy, dx, dw, db, dx_accum=True)
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
    nbytes = rows * D * (x.element_size() + 4 + 8)
    print(f"bwd rows={rows:6d} D={D} {str(xdt):15s} {us:8.1f} us {nbytes / us / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    if "bwd" in sys.argv[1:]:
        for rows, D in ((48000, 768), (96000, 1280), (14304, 768)):
            for xdt in (torch.float32, torch.bfloat16):
                run_bwd(rows, D, xdt)
        sys.exit(0)
    for dt in (torch.bfloat16, torch.float16):
        for rows in (448 * 64, 1500 * 64, 512):
            for add in ((False, True) if dt == torch.bfloat16 else (False,)):
                run(rows, 1280, dt, add)
