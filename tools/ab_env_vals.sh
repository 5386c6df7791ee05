# A/B of two values of an env switch on ONE box (alternating bench runs).
# usage: bash tools/ab_env_vals.sh VAR VAL_A VAL_B [rounds] -> gpurun_out/ab_env_vals.txt
VAR=$1; A=$2; B=$3; R=${4:-3}
rm -f gpurun_out/ab_env_vals.txt
for i in $(seq $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 100 python bench.py --no-cpu-baseline --no-probe --steps 30 > gpurun_out/ab_ev_$v.log 2>&1 || exit 1
    tail -1 gpurun_out/ab_ev_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['value'], d['ms_per_step'])" >> gpurun_out/ab_env_vals.txt
  done
done
