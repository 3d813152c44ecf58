mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
for c in step resonator triple_point scramjet; do
  timeout -k 10 240 python bench.py --config $c --steps 100 --warmup 10 > gpurun_out/bench_$c.log 2>&1 || exit 1
done
timeout -k 10 200 python -m openhyperflow2d_amd run /tmp/none.dat > /dev/null 2>&1
python -m openhyperflow2d_amd deck wedge15 --nx 400 --ny 80 -o gpurun_out/w.dat && timeout -k 10 200 python -m openhyperflow2d_amd run gpurun_out/w.dat --backend gpu --cycles 2 > gpurun_out/cli_gpu.log 2>&1
