cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CASE=${1:-64:fwd+stats} VARIANTS=1 ROUNDS=1 REPS=5
rm -rf gpurun_out/pmc; mkdir -p gpurun_out/pmc
run() { timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $1 --output-format csv -d gpurun_out/pmc/$2 -o p -- python tools/bench_stream3.py > gpurun_out/pmc/$2.log 2>&1; }
run "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES" a && run "TA_DATA_STALLED_BY_TC_CYCLES TA_TOTAL_WAVEFRONTS" b && run "GRBM_GUI_ACTIVE TA_FLAT_READ_LDS_WAVEFRONTS" c
ls gpurun_out/pmc
