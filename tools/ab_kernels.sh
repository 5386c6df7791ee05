# Per-kernel A/B of two builds of libroadrestore on ONE box: rocprofv3
# --kernel-trace of an eager bench run per build, alternating, R rounds.
# usage: bash tools/ab_kernels.sh <other .so> [rounds]
#   -> gpurun_out/abk/{cur,other}_<i>/ (compare with tools/ab_kernels_cmp.py)
OTHER=$1; R=${2:-2}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export RR_PERC_PREFETCH=0
rm -rf gpurun_out/abk && mkdir -p gpurun_out/abk
ARGS="--steps 5 --warmup 3 --repeats 1 --graph 0 --no-cpu-baseline --no-probe"
for i in $(seq $R); do
  for L in cur other; do
    if [ $L = other ]; then export RR_LIB_PATH=$OTHER; else unset RR_LIB_PATH; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abk/${L}_$i -o kt -- python bench.py $ARGS > gpurun_out/abk/${L}_$i.log 2>&1 || exit 1
  done
done
