# cfg5 inference: kernel trace of the 224 pipeline (where restore / judge time goes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/bench_inference.py --images 4096 > gpurun_out/r3ae_inf.json 2> gpurun_out/r3ae_inf.err || exit 1
cat gpurun_out/r3ae_inf.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ae_kt -o kt -- python tools/bench_inference.py --images 2048 > gpurun_out/r3ae_kt.log 2>&1 || exit 1
find gpurun_out/r3ae_kt -name '*.db' | head -3
