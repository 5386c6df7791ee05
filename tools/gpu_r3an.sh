# stream3 dgrad / relu-forward in 128-pixel steps (A/B) + tests under the modes
set -o pipefail
for m in 2 3; do
  RR_S3_MP4_MODE=$m timeout -k 10 300 python -u -m pytest tests/test_stream3_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3an_tests_$m.log 2>&1
  rc=$?; tail -1 gpurun_out/r3an_tests_$m.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_env_multi.sh 3 "RR_S3_MP4_MODE 0 2" "RR_S3_MP4_MODE 0 3" || exit 1
cat gpurun_out/ab_multi.txt
