#!/bin/bash
# triple point (fixed tile 1,50) + headline, for package trees under _ab/<tag> (or head)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for t in "$@"; do
  if [ "$t" = head ]; then d="$R"; else d="$R/_ab/$t"; fi
  (cd "$d" && timeout -k 10 200 python bench.py --config triple_point --steps 100 --warmup 10 --tile ${TILE:-1,50}) > gpurun_out/abtp_${t}.log 2>&1 || exit 1
  (cd "$d" && timeout -k 10 200 python bench.py --steps 2000 --warmup 100) > gpurun_out/abhl_${t}.log 2>&1 || exit 1
done
