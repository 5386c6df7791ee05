set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3c_gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r3c_gpu_tests.log
tail -3 gpurun_out/r3c_gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err || exit 1
cat gpurun_out/r3c_bench.json | head -c 600
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r3c
RR_PERC_PREFETCH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3c/kt -o kt -- python bench.py --steps 5 --warmup 3 --repeats 1 --graph 0 --no-cpu-baseline --no-probe > gpurun_out/prof_r3c/kt.log 2>&1
echo prof rc=$?
