# PMC passes over one tiled-halo conv shape (tools/halo_one.py).
# usage: bash tools/pmc_halo.sh [H:cin:cout]   (on the GPU box; results in gpurun_out/pmch)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CASE=${1:-32:128:128} REPS=5
rm -rf gpurun_out/pmch; mkdir -p gpurun_out/pmch
run() { timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $1 --output-format csv -d gpurun_out/pmch/$2 -o p -- python tools/halo_one.py > gpurun_out/pmch/$2.log 2>&1; }
run "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS" a && \
run "GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_SMEM" b && \
run "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM SQ_WAVES" c
python tools/halo_one.py >> gpurun_out/pmch/time.log 2>&1
ls gpurun_out/pmch
