# full GPU suite, bench, kernel stats of the bench step and of cfg5 inference
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3j_gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r3j_gpu_tests.log
tail -3 gpurun_out/r3j_gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r3j_bench.json 2> gpurun_out/r3j_bench.err || exit 1
head -c 700 gpurun_out/r3j_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r3j
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3j/kt -o kt -- python bench.py --steps 5 --warmup 3 --repeats 1 --graph 0 --no-cpu-baseline --no-probe > gpurun_out/prof_r3j/kt.log 2>&1 || exit 1
echo prof rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3j/inf -o inf -- python tools/bench_inference.py --images 2048 > gpurun_out/prof_r3j/inf.log 2>&1
echo inf prof rc=$?
