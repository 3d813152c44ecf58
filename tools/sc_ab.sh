#!/bin/bash
# A/B of the scalar read-back at the end of a run_steps call on the driver's
# bench command: hf2d_scalars_out kernel (HF2D_SC_KERNEL=1, default) vs a
# device-to-host copy (0), interleaved, 3 reps each.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 1 0; do
    HF2D_SC_KERNEL=$v timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/sc_ab_${v}_${r}.log 2>&1 || exit $?
    python - "$v" "$r" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/sc_ab_%s_%s.log" % (sys.argv[1], sys.argv[2])) if l.startswith("{")][-1]
d = json.loads(line)
print("sc_kernel=%s rep %s: %.2f us/step (%s)" % (sys.argv[1], sys.argv[2], d["ms_per_step"] * 1e3, d["config"]["tile"]), flush=True)
PY
  done
done
