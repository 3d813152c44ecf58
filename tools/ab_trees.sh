#!/bin/bash
# A/B of whole package trees shipped under _ab/<tag>/ (config benches, 1 GPU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for t in "$@"; do
  for c in ${CONFIGS:-step scramjet}; do
    st=100; [ $c = scramjet ] && st=40
    if [ "$t" = head ]; then d="$R"; else d="$R/_ab/$t"; fi
    (cd "$d" && timeout -k 10 200 python bench.py --config $c --steps $st --warmup 10) > gpurun_out/ab_${t}_$c.log 2>&1 || exit 1
  done
done
