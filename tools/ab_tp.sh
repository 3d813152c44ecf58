#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for t in "$@"; do
  if [ "$t" = head ]; then d="$R"; else d="$R/_ab/$t"; fi
  for a in 0 1; do
  (cd "$d" && HF2D_AUTOTUNE=$a timeout -k 10 200 python bench.py --config triple_point --steps 100 --warmup 10) > gpurun_out/abtp_${t}_$a.log 2>&1 || exit 1
  done
done
