"""HBM roofline + PMC calibration: time a device-to-device copy of B bytes and
(under rocprofv3 --pmc FETCH_SIZE WRITE_SIZE) compare the counters with the
known traffic (B read + B written per copy)."""
import sys
import time

import torch


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 80.0
    n = int(mb * 1e6 / 8)
    x = torch.rand(n, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    for _ in range(5):
        y.copy_(x)
    torch.cuda.synchronize()
    reps = 50
    t0 = time.perf_counter()
    for _ in range(reps):
        y.copy_(x)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print("copy %.1f MB: %.2f us, %.2f TB/s (read+write)" % (mb, dt * 1e6, 2 * n * 8 / dt / 1e12), flush=True)


if __name__ == "__main__":
    main()
