#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first
# step that timed out, aborted or crashed (124/137/134/139), carry on after an
# ordinary failure (a failing test).  Usage:
#   bash tools/gpu_step.sh SECONDS LOG -- cmd args...  [ ;; SECONDS LOG -- cmd ... ]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
while [ $# -gt 0 ]; do
  t=$1; log=$2; shift 2; [ "$1" = "--" ] && shift
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != ";;" ]; do cmd+=("$1"); shift; done
  [ "$1" = ";;" ] && shift
  timeout -k 10 "$t" "${cmd[@]}" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "[gpu_step] ${cmd[*]:0:4} -> rc=$rc"
  case $rc in 124|137|134|139) echo "[gpu_step] stopping after rc=$rc"; exit $rc ;; esac
done
