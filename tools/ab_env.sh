#!/bin/bash
# A/B of bench.py on this tree between two values of one environment
# variable, interleaved (A B A B), one time limit per run; the first failure
# ends it:
#   bash tools/ab_env.sh VAR VALUE_A VALUE_B TAG bench.py-args...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
var=$1; va=$2; vb=$3; tag=$4; shift 4
for rep in 1 2; do
  for v in "$va" "$vb"; do
    env "$var=$v" timeout -k 10 300 python bench.py "$@" > "gpurun_out/abe_${tag}_${v}_${rep}.log" 2>&1 || exit 1
    grep -o '"ms_per_step": [0-9.]*' "gpurun_out/abe_${tag}_${v}_${rep}.log" | sed "s/^/$tag $var=$v rep$rep /"
  done
done
