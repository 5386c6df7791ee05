# PMC passes over the streaming conv (tools/bench_stream3.py, one case).
# usage: bash tools/pmc_stream3.sh [CASE]   (on the GPU box; results in gpurun_out/pmc)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CASE=${1:-64:fwd+stats} VARIANTS=stream3=1 ROUNDS=1 REPS=5
rm -rf gpurun_out/pmc; mkdir -p gpurun_out/pmc
run() { timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $1 --output-format csv -d gpurun_out/pmc/$2 -o p -- python tools/bench_stream3.py > gpurun_out/pmc/$2.log 2>&1; }
run "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS" a && \
run "GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_SMEM" b && \
run "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM SQ_WAVES" c && \
run "FETCH_SIZE" d && run "WRITE_SIZE" e
ls gpurun_out/pmc
