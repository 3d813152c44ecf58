#!/bin/bash
# Launcher (cf. the reference's bin/OpenHyperFLOW2D.sh <Project> [nhosts], which
# runs mpiexec over NHOSTS x cores): one process per MI355X through torchrun.
#   OpenHyperFLOW2D.sh <Project|deck.dat> [ngpus] [extra run options]
# <Project> resolves to <Project>.dat in the current directory.  Outputs go next
# to the deck (reference behaviour); ngpus defaults to 1.
set -euo pipefail
if [ $# -lt 1 ]; then
  echo "Usage: $0 <Project|deck.dat> [ngpus] [run options]" >&2
  exit 2
fi
deck="$1"
shift
[ -f "$deck" ] || deck="$deck.dat"
[ -f "$deck" ] || { echo "deck not found: $1" >&2; exit 2; }
ngpus=1
if [ $# -gt 0 ] && [[ "$1" =~ ^[0-9]+$ ]]; then
  ngpus="$1"
  shift
fi
here="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
export PYTHONPATH="$here${PYTHONPATH:+:$PYTHONPATH}"
export HSA_ENABLE_IPC_MODE_LEGACY="${HSA_ENABLE_IPC_MODE_LEGACY:-0}"
if [ "$ngpus" -le 1 ]; then
  exec python3 -m openhyperflow2d_amd run "$deck" "$@"
fi
exec python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$ngpus" --master-addr 127.0.0.1 \
  --master-port "${HF2D_MASTER_PORT:-29613}" -m openhyperflow2d_amd run "$deck" "$@"
