# halo wgrad: MA / PF variants per layer, tests, same-box step A/B against ablib/base.so
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_swgrad_gpu.py -q -x -k "wgrad" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3ag_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3ag_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_wgrad_ma.py > gpurun_out/r3ag_ab_wgrad.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3ag_ab_wgrad.jsonl
bash tools/ab_libs.sh ablib/base.so 3 || exit 1
cat gpurun_out/ab_libs.txt
