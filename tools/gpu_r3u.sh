set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r3u
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3u/inf -o inf -- python tools/bench_inference.py --images 2048 > gpurun_out/prof_r3u/inf.log 2>&1
echo inf prof rc=$?
