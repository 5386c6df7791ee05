set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_conv3r_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3q_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3q_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ab_conv3r.py RR_CONV3R_PERSIST=1,0,1,0 > gpurun_out/r3q_ab.jsonl 2>&1 || exit 1
tail -1 gpurun_out/r3q_ab.jsonl
SET=224 timeout -k 10 200 python tools/ab_conv3r.py RR_CONV3R_PERSIST=1,0 > gpurun_out/r3q_ab224.jsonl 2>&1 || exit 1
tail -1 gpurun_out/r3q_ab224.jsonl
