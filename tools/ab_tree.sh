#!/bin/bash
# A/B of bench.py between this tree and another built tree on one GPU box,
# interleaved (A B A B), one time limit per run; the first failure ends it:
#   bash tools/ab_tree.sh OTHER_TREE_DIR TAG bench.py-args...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
other=$1; tag=$2; shift 2
for rep in 1 2; do
  for t in "$other" .; do
    name=$( [ "$t" = "." ] && echo head || echo other )
    (cd "$t" && timeout -k 10 300 python bench.py "$@") > "gpurun_out/abt_${tag}_${name}_${rep}.log" 2>&1 || exit 1
    grep -o '"ms_per_step": [0-9.]*' "gpurun_out/abt_${tag}_${name}_${rep}.log" | sed "s/^/$tag $name rep$rep /"
  done
done
