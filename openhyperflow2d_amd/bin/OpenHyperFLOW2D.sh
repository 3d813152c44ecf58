#!/bin/bash
# Launcher (cf. the reference's bin/OpenHyperFLOW2D.sh <Project> [nhosts], which
# runs mpiexec over NHOSTS x cores): N processes of the native bin/hf2d, one
# strip rank each (one per MI355X with the GPU backend), no Python.
#   OpenHyperFLOW2D.sh <Project|deck.dat> [nranks] [hf2d options]
# <Project> resolves to <Project>.dat in the current directory; outputs go to
# the current directory (reference behaviour) unless --outdir is given.  The
# ranks meet at 127.0.0.1:$HF2D_MASTER_PORT (default 29613) through the
# RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* variables torchrun also sets.
set -uo pipefail
if [ $# -lt 1 ]; then
  echo "Usage: $0 <Project|deck.dat> [nranks] [hf2d options]" >&2
  exit 2
fi
deck="$1"
shift
[ -f "$deck" ] || deck="$deck.dat"
[ -f "$deck" ] || { echo "deck not found: $deck" >&2; exit 2; }
n=1
if [ $# -gt 0 ] && [[ "$1" =~ ^[0-9]+$ ]]; then
  n="$1"
  shift
fi
[ "$n" -ge 1 ] || n=1
here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
bin="${HF2D_BIN:-$here/hf2d}"
[ -x "$bin" ] || bin="$here/hf2d_cpu"
[ -x "$bin" ] || { echo "native binary not built (python -c 'import openhyperflow2d_amd._build as b; b.build()')" >&2; exit 2; }
export HSA_ENABLE_IPC_MODE_LEGACY="${HSA_ENABLE_IPC_MODE_LEGACY:-0}"
if [ "$n" -eq 1 ]; then
  exec "$bin" "$@" "$deck"
fi
port="${HF2D_MASTER_PORT:-29613}"
pids=()
for ((r = 0; r < n; r++)); do
  RANK=$r WORLD_SIZE=$n LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$port "$bin" "$@" "$deck" &
  pids+=($!)
done
# a failed rank makes the others fail at their next collective; keep the
# first non-zero status
rc=0
for p in "${pids[@]}"; do
  wait "$p"
  s=$?
  [ $rc -ne 0 ] || rc=$s
done
exit $rc
