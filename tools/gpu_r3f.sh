timeout -k 10 500 python -u -m pytest tests/test_conv3r_gpu.py tests/test_stream3_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3f_conv3r.log 2>&1
echo "tests rc=$?" >> gpurun_out/r3f_conv3r.log
tail -2 gpurun_out/r3f_conv3r.log
timeout -k 10 400 python tools/ab_conv3r.py RR_CONV3R_WG=4,8 RR_IGEMM_DBG=0,1,8 > gpurun_out/r3f_ab.jsonl 2>&1
tail -1 gpurun_out/r3f_ab.jsonl
