# A/B of two builds of libroadrestore on ONE box: alternating bench runs
# (single-run noise ~0.7%; box-to-box spread is larger, so compare in-call).
# usage: bash tools/ab_libs.sh <other .so> [rounds]   -> gpurun_out/ab_libs.txt
OTHER=$1; R=${2:-3}
rm -f gpurun_out/ab_libs.txt
for i in $(seq $R); do
  for L in cur other; do
    if [ $L = other ]; then export RR_LIB_PATH=$OTHER; else unset RR_LIB_PATH; fi
    timeout -k 10 100 python bench.py --no-cpu-baseline --no-probe --steps 30 > gpurun_out/ab_$L.log 2>&1 || exit 1
    tail -1 gpurun_out/ab_$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['value'], d['ms_per_step'])" >> gpurun_out/ab_libs.txt
  done
done
