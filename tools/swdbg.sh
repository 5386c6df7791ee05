cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1 5 2 3 7; do
  CASE=64:wgrad VARENV=RR_SW_DBG VARIANTS=$v ROUNDS=1 REPS=10 timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/swdbg/$v -o k -- python tools/bench_stream3.py > gpurun_out/swdbg/$v.log 2>&1 || exit 1
done
