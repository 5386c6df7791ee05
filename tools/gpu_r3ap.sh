# conv3r half-width column blocks (RR_CONV3R_BCDIV=2): tests, per-layer A/B, graph-step A/B
set -o pipefail
RR_CONV3R_BCDIV=2 timeout -k 10 400 python -u -m pytest tests/test_conv3r_gpu.py -q -x -k "not selected" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3ap_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r3ap_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_conv3r.py RR_CONV3R_BCDIV=0,2 > gpurun_out/r3ap_ab.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3ap_ab.jsonl | tail -1
bash tools/ab_env_multi.sh 3 "RR_CONV3R_BCDIV 0 2" || exit 1
cat gpurun_out/ab_multi.txt
