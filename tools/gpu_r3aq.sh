# round-3 evidence: full GPU suite, bench, profile passes (kernel stats, HBM traffic, MFMA busy)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3aq_gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r3aq_gpu_tests.log
tail -3 gpurun_out/r3aq_gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r3aq_bench.json 2> gpurun_out/r3aq_bench.err || exit 1
head -c 400 gpurun_out/r3aq_bench.json
bash tools/profile_round.sh r3aq > gpurun_out/r3aq_prof.log 2>&1
echo "prof rc=$?"
