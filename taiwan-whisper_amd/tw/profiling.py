"""Per-launch HIP-event timing of one kernel family inside a timed region (the roofline leg of
bench.py).  Events are recorded on the stream the kernels are launched on (torch's current
stream, which every tw op uses)."""
from __future__ import annotations

import torch


class KernelTimer:
    active = None   # the KernelTimer currently collecting, or None

    def __init__(self, *families: str):
        self.families = families
        self.family = families[0]
        self.records = {f: [] for f in families}   # family -> [(start_event, end_event, work, bytes)]

    def __enter__(self):
        KernelTimer.active = self
        return self

    def __exit__(self, *exc):
        KernelTimer.active = None

    @staticmethod
    def wrap(family, work, launch, nbytes=0.0):
        """work = algorithmic flops (or bytes) of the launch; nbytes = its algorithmic HBM bytes (every
        operand read once, every output written once), for the traffic-vs-algorithm ratio."""
        t = KernelTimer.active
        if t is None or family not in t.records:
            return launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = launch()
        e1.record()
        t.records[family].append((e0, e1, work, nbytes))
        return r

    def summary(self, family=None):
        torch.cuda.synchronize()
        rec = self.records[family or self.family]
        ms = [r[0].elapsed_time(r[1]) for r in rec]
        work = [r[2] for r in rec]
        nbytes = sum(r[3] for r in rec)
        n = len(ms)
        if n == 0:
            return None
        tot_ms, tot_w = sum(ms), sum(work)
        return dict(launches=n, avg_ms=tot_ms / n, total_ms=tot_ms, avg_work=tot_w / n,
                    rate=tot_w / (tot_ms * 1e-3), avg_bytes=nbytes / n)
