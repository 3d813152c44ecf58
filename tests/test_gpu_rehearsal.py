"""Multi-process rehearsals of the multi-rank paths on one GPU: N rank
processes share the device (gloo host collectives, IPC-mapped xGMI mailbox
halos), as the driver's N-GPU runs do with one device each.

* the Python driver (DistributedSimulation.run: outer cycles, strip outputs,
  checkpoints) at 2 and 4 ranks writes the same bytes as one process
  (tools/rehearse_run.py);
* bench.py --gpus 4 (HF2D_BENCH_SHARED_GPU=1) completes and reports one JSON
  line with the validated mailbox transport -- the round-6 deadlock (ranks in
  different collectives after rank-local step-graph choices) would hang here."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(n, args, env=None, timeout=100):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    e = dict(os.environ, **(env or {}))
    return subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("nranks", [2, 4])
def test_python_driver_ranks_match_one(gpu, tmp_path, nranks):
    tool = os.path.join(ROOT, "tools", "rehearse_run.py")
    one = subprocess.run([sys.executable, tool, str(tmp_path / "one")], cwd=ROOT, capture_output=True, text=True,
                         timeout=100)
    assert one.returncode == 0, one.stdout[-2000:] + one.stderr[-2000:]
    r = _torchrun(nranks, [tool, str(tmp_path / "n")])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "transport p2p" in r.stdout
    c = subprocess.run([sys.executable, tool, "--compare", str(tmp_path / "one"), str(tmp_path / "n")], cwd=ROOT,
                       capture_output=True, text=True, timeout=60)
    assert c.returncode == 0, c.stdout


def test_bench_four_ranks_on_one_gpu(gpu):
    r = _torchrun(4, ["bench.py", "--gpus", "4", "--steps", "10", "--warmup", "3"],
                  env={"HF2D_BENCH_SHARED_GPU": "1", "HF2D_BENCH_STACKS": "30"})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["steps"] == 10 and d["rehearsal_shared_gpu"] is True
    assert d["config"]["transport"] == "p2p" and d["config"]["p2p_validated"] is True
