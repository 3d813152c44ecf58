#!/bin/bash
# One entry point for the GPU-box jobs (run through gpurun from the repo root):
#
#   bash tools/gpu_suite.sh tests            pytest -m gpu + smoke()
#   bash tools/gpu_suite.sh bench [STEPS]    headline bench.py (1 GPU)
#   bash tools/gpu_suite.sh configs          bench.py for every BASELINE config
#   bash tools/gpu_suite.sh prof [ARGS...]   rocprofv3 kernel trace + stats of bench.py ARGS
#   bash tools/gpu_suite.sh pmc CTRS [ARGS]  one rocprofv3 --pmc pass (counters in CTRS, space separated)
#   bash tools/gpu_suite.sh strips           one-GPU proxies of the 8- and 4-GPU headline strips
#                                            (250 / 500 columns + fused xGMI mailbox exchange) and
#                                            the same strips alone on one rank
#   bash tools/gpu_suite.sh all              tests && bench && prof
#
# Every GPU step has its own time limit and the steps are chained with &&:
# the first failure ends the job (no retries).  Logs go to gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
mode=${1:-all}
shift || true

run_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 &&
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
}
run_bench() {
  timeout -k 10 300 python bench.py --steps "${1:-2000}" --warmup 200 > gpurun_out/bench1.log 2>&1
}
run_configs() {
  for c in step resonator triple_point scramjet; do
    timeout -k 10 240 python bench.py --config $c --steps 100 --warmup 10 > gpurun_out/bench_$c.log 2>&1 || return 1
  done
}
run_strips() {
  # one strip of the 8 / 4-rank headline split alone and with the mailbox exchange (loopback)
  for n in 8 4; do
    timeout -k 10 240 python tools/exchange_loopback.py --config wedge15 --ranks $n >> gpurun_out/loopback.jsonl \
      2> gpurun_out/loopback_$n.err || return 1
  done
}
run_prof() {
  local tag=${PROF_TAG:-bench}
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag" -o run \
     -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/prof_$tag.log" 2>&1)
}
run_pmc() {
  local ctrs=$1
  shift
  local tag=${PROF_TAG:-pmc}
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_$tag" -o run \
     -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/pmc_$tag.log" 2>&1)
}

case $mode in
  tests) run_tests ;;
  bench) run_bench "$@" ;;
  configs) run_configs ;;
  strips) run_strips ;;
  prof) run_prof "$@" ;;
  pmc) run_pmc "$@" ;;
  all) run_tests && run_bench && run_prof --steps 500 --warmup 50 ;;
  *) echo "unknown mode $mode" >&2; exit 2 ;;
esac
