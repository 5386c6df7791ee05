# conv3r stall counters: cfg3 layers (B=512) and cfg5 layers (SET=224, B=64)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_r3m
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
REPS=3 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_r3m/a -o a -- python tools/ab_conv3r.py > gpurun_out/pmc_r3m/a.log 2>&1 || exit 1
echo a ok
SET=224 REPS=3 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_r3m/b -o b -- python tools/ab_conv3r.py > gpurun_out/pmc_r3m/b.log 2>&1 || exit 1
echo b ok
SET=224 timeout -k 10 120 python tools/ab_conv3r.py > gpurun_out/r3m_ab224.jsonl 2>&1
tail -1 gpurun_out/r3m_ab224.jsonl
