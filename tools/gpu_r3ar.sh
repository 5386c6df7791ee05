# graph-step A/B of the streaming-kernel eligibility switches
set -o pipefail
bash tools/ab_env_multi.sh 2 "RR_STREAM1_MINP 131072 32768" "RR_SWGRAD 1 0" "RR_STREAM1 1 0" || exit 1
cat gpurun_out/ab_multi.txt
