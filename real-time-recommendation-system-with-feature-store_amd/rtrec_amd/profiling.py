"""Live per-kernel timing with HIP events (bench.py's roofline numbers).

``TIMER.region(name, flops=..., bytes_=...)`` brackets one ABI call with two
events recorded on the stream the kernels are launched on (torch's current
stream, which every wrapper passes to the C ABI), and records the algorithmic
work of that call. Disabled (zero overhead beyond a flag check) unless a
benchmark enables it for a chosen set of names.
"""
from __future__ import annotations

from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, Iterable, Optional

import torch


class KernelTimer:
    def __init__(self):
        self.enabled = False
        self.names: Optional[set] = None
        self.spacer = 0
        self.records = defaultdict(list)

    def enable(self, names: Optional[Iterable[str]] = None, spacer_cycles: int = 0):
        """``spacer_cycles`` > 0 enqueues a GPU spin of that many cycles before each
        timed region, so the host's submission of the call (ctypes, argument
        structs) completes while the GPU is still busy: the start event then
        fires right before the kernel instead of when the host gets there."""
        self.enabled = True
        self.names = set(names) if names is not None else None
        self.spacer = int(spacer_cycles)
        self.records.clear()

    def disable(self):
        self.enabled = False

    @contextmanager
    def region(self, name: str, flops: float = 0.0, bytes_: float = 0.0, device=None):
        if not self.enabled or (self.names is not None and name not in self.names):
            yield
            return
        st = torch.cuda.current_stream(device)
        if self.spacer > 0:
            torch.cuda._sleep(self.spacer)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        try:
            yield
        finally:
            e1.record(st)
            self.records[name].append((e0, e1, flops, bytes_))

    def summary(self) -> Dict[str, dict]:
        torch.cuda.synchronize()
        out = {}
        for name, recs in self.records.items():
            ms = sum(a.elapsed_time(b) for a, b, _, _ in recs)
            out[name] = {"count": len(recs), "total_ms": ms, "avg_ms": ms / max(1, len(recs)),
                         "flops": sum(r[2] for r in recs), "bytes": sum(r[3] for r in recs)}
        return out


TIMER = KernelTimer()
