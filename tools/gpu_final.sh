#!/bin/bash
# end-of-session check: GPU suite + smoke, headline (2000 steps and the driver's 20-step command), configs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
bash tools/gpu_suite.sh tests && bash tools/gpu_suite.sh bench 2000 &&
for k in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/short_$k.log 2>&1 || exit 1
done && bash tools/gpu_suite.sh configs
