# re-run the round's failing GPU tests; a clean (no side-stream prefetch) kernel profile of the step
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_bf16_model_gpu.py tests/test_models_gpu.py tests/test_lifetime_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3k_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r3k_tests.log
tail -4 gpurun_out/r3k_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r3k
RR_PERC_PREFETCH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3k/kt -o kt -- python bench.py --steps 5 --warmup 3 --repeats 1 --graph 0 --no-cpu-baseline --no-probe > gpurun_out/prof_r3k/kt.log 2>&1
echo prof rc=$?
