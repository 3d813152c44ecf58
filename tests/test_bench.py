"""bench.py driver contract: ``--gpus N`` runs N ranks (spawned by bench.py
itself when there is no torchrun environment), prints one JSON line from
rank 0, and the strip run reaches the same dt as one rank (gloo, CPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--backend", "cpu", "--nx", "120", "--ny", "30", "--steps", "6", "--warmup", "2"]


def _run(extra, env_over=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_over or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + ARGS + extra, env=env,
                       capture_output=True, text=True, timeout=600)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, lines, r.stderr


def test_bench_gpus_n_launches_n_ranks(hf):
    rc1, l1, err1 = _run([])
    rc4, l4, err4 = _run(["--gpus", "4"])
    assert rc1 == 0 and len(l1) == 1, err1
    assert rc4 == 0 and len(l4) == 1, err4
    one, four = json.loads(l1[0]), json.loads(l4[0])
    assert one["ranks"] == 1 and four["ranks"] == 4
    assert four["config"]["parallelism"] == "strip4"
    assert four["final_dt"] == one["final_dt"] and four["final_time"] == one["final_time"]
    assert four["steps"] == 6 and four["warmup"] == 2


def test_bench_world_size_mismatch_fails_loudly(hf):
    rc, lines, err = _run(["--gpus", "2"], {"WORLD_SIZE": "1"})
    assert rc != 0 and not lines
    assert "WORLD_SIZE=1" in err
