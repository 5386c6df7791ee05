# graph-replay kernel trace (idle time between kernels in the captured step) and
# a stall-counter pass over the eager bench (where the waves of each kernel wait)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export RR_PERC_PREFETCH=0
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3ah_graph -o g -- python bench.py --steps 20 --warmup 5 --repeats 1 --graph 1 --no-cpu-baseline --no-probe > gpurun_out/r3ah_graph.log 2>&1 || exit 1
tail -c 300 gpurun_out/r3ah_graph.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/r3ah_stalls -o s -- python bench.py --steps 5 --warmup 3 --repeats 1 --graph 0 --no-cpu-baseline --no-probe > gpurun_out/r3ah_stalls.log 2>&1 || exit 1
find gpurun_out/r3ah_graph gpurun_out/r3ah_stalls -name '*.db'
