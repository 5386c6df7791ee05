# re-validate scheduling / grid switches in the graph-captured step
set -o pipefail
bash tools/ab_env_multi.sh 2 "RR_WGRAD_SIDE_STREAM 0 1" "RR_WGRAD_HALO_WGS 512 1024" "RR_WGRAD_HALO_WGS 512 256" "RR_CONV3R_WG 0 8" "RR_PERC_PREFETCH 1 0" "RR_XCD_MAP 1 0" || exit 1
cat gpurun_out/ab_multi.txt
