cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcx
for v in 0 1; do
  RR_XCD_MAP=$v CASE=32:128:128 REPS=3 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcx/f$v -o p -- python tools/halo_one.py > gpurun_out/pmcx/f$v.log 2>&1 || exit 1
done
