# Several env-switch A/Bs on ONE box, each as alternating bench runs (graph step):
# usage: bash tools/ab_env_multi.sh ROUNDS "VAR A B" ["VAR A B" ...] -> gpurun_out/ab_multi.txt
R=$1; shift
rm -f gpurun_out/ab_multi.txt
for spec in "$@"; do
  set -- $spec
  VAR=$1; A=$2; B=$3
  for i in $(seq $R); do
    for v in $A $B; do
      env $VAR=$v timeout -k 10 100 python bench.py --no-cpu-baseline --no-probe --steps 30 > gpurun_out/ab_m.log 2>&1 || exit 1
      tail -1 gpurun_out/ab_m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['value'], d['ms_per_step'])" >> gpurun_out/ab_multi.txt
    done
  done
done
