# conv3r ALT (4-wave, double-buffered halo, 128x32 wave tiles) tests + per-layer A/B; cfg5 kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_conv3r_gpu.py -q -x -k "alt or selected" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3af_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3af_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_conv3r.py RR_CONV3R_ALT=0,1 > gpurun_out/r3af_ab_alt.jsonl 2>&1 || exit 1
tail -3 gpurun_out/r3af_ab_alt.jsonl
bash tools/gpu_r3ae.sh
