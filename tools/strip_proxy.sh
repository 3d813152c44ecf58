#!/bin/bash
# One-GPU proxies of the 4-strip resonator and the 8-strip scramjet: wall time + rocprofv3 kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 300 python tools/strip_proxy.py "$@" > gpurun_out/proxy_$tag.log 2>&1 || return 1
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/proxyprof_$tag" -o run \
     -- python3 "$R/tools/strip_proxy.py" "$@" > "$R/gpurun_out/proxyprof_$tag.log" 2>&1)
}
export GPU_MAX_HW_QUEUES=16
run reso4 --config resonator --ranks 4 --steps 60 && run reso4x --config resonator --ranks 4 --steps 60 --nofuse && \
run reso1 --config resonator --ranks 1 --steps 60 && run scram8 --config scramjet --ranks 8 --steps 12 --warmup 12
