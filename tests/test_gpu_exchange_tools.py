"""The one-GPU exchange measurement tool (tools/exchange_loopback.py): a strip
timed alone and as rank r of N over the xGMI mailbox transport looped back on
itself, and --trace, the fused tail's phase clocks (HF2D_FX_SKIP bit 4, read
back through DeviceSolver.fx_trace).  Timing-only instrumentation: the run
must still produce a finite exchange cost and one clock per tail phase."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("config,ranks", [("wedge15", 4), ("resonator", 4)])
def test_exchange_loopback_trace_reports_every_tail_phase(gpu, config, ranks):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "exchange_loopback.py"), "--config", config,
                        "--ranks", str(ranks), "--steps", "100", "--warmup", "20", "--repeat", "1", "--trace"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["fused"] and rec["loopback_us"][0] > 0 and rec["alone_us"][0] > 0
    t = rec["tail_us"]
    assert set(t) == {"drain", "count", "dt_min", "dt_publish", "flags", "wait_fold", "store", "total"}
    assert t["total"] > 0 and all(v >= 0 for v in t.values()), t
    assert abs(sum(v for k, v in t.items() if k != "total") - t["total"]) < 0.5 * t["total"] + 0.5, t
