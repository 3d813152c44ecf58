set -o pipefail
cd ${GRAFT_REPO_ROOT}
export TMPDIR=/tmp
for t in _ab0 .; do
  n=$( [ "$t" = "." ] && echo head || echo other )
  (cd $t && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${GRAFT_REPO_ROOT}/gpurun_out/prof_$n -o run -- python3 bench.py --config scramjet --steps 100 --warmup 10) > gpurun_out/prof_$n.log 2>&1 || exit 1
done
