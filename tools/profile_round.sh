# rocprofv3 evidence for the bench (run on the GPU box from the repo root):
#   1. --kernel-trace --stats of an eager bench run  -> per-kernel summary CSV
#   2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes -> HBM bytes / launch
#   3. MFMA busy cycles + GRBM_GUI_ACTIVE (one pass) -> MFMA utilisation / clock per kernel
# usage: bash tools/profile_round.sh <tag>   (outputs profiles/<tag>_*)
set -e
TAG=${1:-r1}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof_$TAG
# per-kernel durations without the perceptual-target prefetch running
# concurrently on its side stream (bench.py's probe does the same)
export RR_PERC_PREFETCH=0
rm -rf $OUT && mkdir -p $OUT
ARGS="--steps 5 --warmup 3 --repeats 1 --graph 0 --no-cpu-baseline --no-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python bench.py $ARGS > $OUT/kt.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o f -- python bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o w -- python bench.py $ARGS > $OUT/write.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $OUT/mfma -o m -- python bench.py $ARGS > $OUT/mfma.log 2>&1
find $OUT -name "*.db" -o -name "*stats.csv" | head -20
