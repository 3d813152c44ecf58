#!/bin/bash
# A/B/C... of bench.py on this tree over several values of one environment
# variable, interleaved (v1 v2 v3 v1 v2 v3 ...), one time limit per run; the
# first failure ends it:
#   bash tools/ab_envn.sh VAR TAG "v1 v2 v3" REPS bench.py-args...
# prints one "TAG VAR=v repK ms_per_step" line per run; logs in gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
var=$1; tag=$2; vals=$3; reps=$4; shift 4
for rep in $(seq 1 "$reps"); do
  for v in $vals; do
    env "$var=$v" timeout -k 10 300 python bench.py "$@" > "gpurun_out/abn_${tag}_${v}_${rep}.log" 2>&1 || exit 1
    grep -o '"ms_per_step": [0-9.]*' "gpurun_out/abn_${tag}_${v}_${rep}.log" | sed "s/^/$tag $var=$v rep$rep /"
  done
done
