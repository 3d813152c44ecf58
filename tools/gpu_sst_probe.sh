set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stability_probe.py scramjet 6000 400 --steps 3000 --chunk 300 --kw turbulence=6 > gpurun_out/sst_probe_a.log 2>&1
timeout -k 10 300 python -u tools/stability_probe.py scramjet 6000 400 --steps 3000 --chunk 300 --kw turbulence=6 --set ViscousCFL=0.4 > gpurun_out/sst_probe_b.log 2>&1
exit 0
