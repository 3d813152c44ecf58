set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/tile_trace.log
timeout -k 10 120 python tools/tile_trace.py --nx 250 >> gpurun_out/tile_trace.log 2>&1 && \
timeout -k 10 120 python tools/tile_trace.py --nx 250 --cpt 1 --tj 16 >> gpurun_out/tile_trace.log 2>&1 && \
timeout -k 10 120 python tools/tile_trace.py --nx 2000 >> gpurun_out/tile_trace.log 2>&1
