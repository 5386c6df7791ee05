# conv3r row-segment tiles: per-op tests, the 64^2 layer A/B, cfg5 inference
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_conv3r_gpu.py tests/test_stream3_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3i_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r3i_tests.log; tail -3 gpurun_out/r3i_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_conv3r.py RR_CONV3R_WG=4,8 > gpurun_out/r3i_ab.jsonl 2>&1 || exit $?
tail -2 gpurun_out/r3i_ab.jsonl
timeout -k 10 300 python tools/bench_inference.py --images 4096 > gpurun_out/r3i_inf_bf16.json 2> gpurun_out/r3i_inf.err || exit $?
cat gpurun_out/r3i_inf_bf16.json
