"""Wall-clock step timing and rocprofv3 result summaries."""
from __future__ import annotations

import sqlite3
import time
from typing import List, Tuple


class StepTimer:
    """Times blocks of solver steps with device synchronisation on both
    sides; reports Mcells*it/s like the reference's 'average speed' line."""

    def __init__(self, sim):
        self.sim = sim
        self.samples: List[Tuple[int, float]] = []

    def _sync(self):
        sync = getattr(self.sim.solver, "synchronize", None)
        if sync:
            sync()

    def run(self, n: int) -> float:
        self._sync()
        t0 = time.perf_counter()
        self.sim.step(n)
        self._sync()
        dt = time.perf_counter() - t0
        self.samples.append((n, dt))
        return dt

    def mcells_per_s(self) -> float:
        nx, ny = self.sim.shape
        steps = sum(n for n, _ in self.samples)
        secs = sum(t for _, t in self.samples)
        return nx * ny * steps / secs / 1e6 if secs else 0.0


def rocprof_kernel_table(db_path: str) -> List[Tuple[str, int, float, float, float]]:
    """(kernel, calls, total_us, avg_us, percent) from a rocprofv3 results .db."""
    con = sqlite3.connect(db_path)
    try:
        rows = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
        return [(n.split("(")[0].replace("void ", ""), int(c), float(t), float(a), float(p)) for n, c, t, a, p in rows]
    finally:
        con.close()
