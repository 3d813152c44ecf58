set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_old.log
for r in 1 2 3; do
(cd _abold && timeout -k 10 120 python bench.py --steps 2000 --warmup 200) >> gpurun_out/ab_old.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 2000 --warmup 200 >> gpurun_out/ab_old.log 2>&1 || exit 1
done
