#!/bin/bash
# Driver command with the autotune (which now also decides step graphs on /
# off), three runs, plus fixed geometry with graphs forced on / off via the
# autotune-free path.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/graph_ab_$r.log 2>&1 || exit $?
  python - "$r" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/graph_ab_%s.log" % sys.argv[1]) if l.startswith("{")][-1])
print("driver run %s: %.2f us/step, graphs %s, %s" % (sys.argv[1], d["ms_per_step"] * 1e3, d["config"]["step_graphs"],
                                                     d["config"]["autotune"][-120:]), flush=True)
PY
done
