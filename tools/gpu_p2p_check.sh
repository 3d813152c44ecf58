set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "p2p or virtual or graphs" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_p2p.log 2>&1 && \
timeout -k 10 120 python tools/p2p_probe.py --ranks 2 > gpurun_out/p2p_probe.log 2>&1 && \
timeout -k 10 120 python tools/p2p_probe.py --ranks 2 --nofuse >> gpurun_out/p2p_probe.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_p2pf -o p2p -- python tools/p2p_probe.py --ranks 2 --steps 300 > gpurun_out/p2p_prof.log 2>&1
