#!/bin/bash
# A/B of an environment knob on one GPU box:
#   bash tools/ab_env.sh VAR "VAL_A VAL_B" TAG bench.py-args...
# Each run has its own time limit; the first failure ends the job.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
var=$1; vals=$2; tag=$3; shift 3
for v in $vals; do
  env "$var=$v" timeout -k 10 240 python bench.py "$@" > "gpurun_out/ab_${tag}_${var}_${v}.log" 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' "gpurun_out/ab_${tag}_${var}_${v}.log" | sed "s/^/$tag $var=$v /"
done
