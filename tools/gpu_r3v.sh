set -o pipefail
RR_CONV3R_SEGWG=8 timeout -k 10 400 python -u -m pytest tests/test_conv3r_gpu.py -k "seg or ex_" -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3v_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3v_tests.log; [ $rc -eq 0 ] || exit $rc
SET=224 timeout -k 10 300 python tools/ab_conv3r.py RR_CONV3R_SEGWG=4,8,4,8 > gpurun_out/r3v_ab224.jsonl 2>&1 || exit 1
tail -1 gpurun_out/r3v_ab224.jsonl
