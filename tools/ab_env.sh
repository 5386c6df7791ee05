# A/B of an env switch on ONE box: alternating bench runs.
# usage: bash tools/ab_env.sh VAR [rounds]  (VAR=0 vs VAR=1) -> gpurun_out/ab_env.txt
VAR=$1; R=${2:-3}
rm -f gpurun_out/ab_env.txt
for i in $(seq $R); do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 100 python bench.py --no-cpu-baseline --no-probe --steps 30 > gpurun_out/ab_env_$v.log 2>&1 || exit 1
    tail -1 gpurun_out/ab_env_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['value'], d['ms_per_step'])" >> gpurun_out/ab_env.txt
  done
done
