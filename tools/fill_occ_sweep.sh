set -e
for spec in "step 0" "step 4" "resonator 0" "resonator 3" "scramjet 0" "scramjet 2"; do
  set -- $spec
  timeout -k 10 200 python bench.py --config $1 --steps 100 --warmup 10 --fill-occ $2 > gpurun_out/occ_$1_$2.log 2>&1
  echo "$1 occ=$2 $(tail -1 gpurun_out/occ_$1_$2.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"])')"
done
