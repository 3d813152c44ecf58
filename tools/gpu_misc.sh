#!/bin/bash
# short-K headline (the driver's --steps 20 --warmup 5), scramjet repeat, strip proxies
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for k in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/short_$k.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --config scramjet --steps 100 --warmup 10 > gpurun_out/scram_rep.log 2>&1 || exit 1
bash tools/strip_proxy.sh
