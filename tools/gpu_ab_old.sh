set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_old.log
for c in scramjet resonator; do
for r in 1 2; do
(cd _abold && timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10) >> gpurun_out/ab_old.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10 >> gpurun_out/ab_old.log 2>&1 || exit 1
done
done
