set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_conv3r_gpu.py tests/test_stream1_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3x_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3x_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_inference.py --images 4096 > gpurun_out/r3x_inf_bf16.json 2> gpurun_out/r3x_inf.err || exit 1
cat gpurun_out/r3x_inf_bf16.json
