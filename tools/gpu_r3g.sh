timeout -k 10 600 python tools/ab_conv3r.py RR_IGEMM_DBG=0,16,32,48,64,1,49,56 > gpurun_out/r3g_ab.jsonl 2>&1
tail -1 gpurun_out/r3g_ab.jsonl
