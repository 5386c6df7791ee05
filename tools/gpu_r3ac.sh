# pack-kernel vectorisation + halo wgrad MA=4 tiles: per-op tests, A/B, bench
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_swgrad_gpu.py -q -x -k "pack or wgrad" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3ac_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3ac_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_wgrad_ma.py > gpurun_out/r3ac_ab_wgrad_ma.jsonl 2>&1 || exit 1
cat gpurun_out/r3ac_ab_wgrad_ma.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r3ac_bench.json 2> gpurun_out/r3ac_bench.err || exit 1
head -c 300 gpurun_out/r3ac_bench.json
