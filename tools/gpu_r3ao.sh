# graph-step re-validation of fusion / kernel-choice switches decided on eager runs
set -o pipefail
bash tools/ab_env_multi.sh 2 "RR_MFMA_PRIO 1 0" "RR_FUSE_BNBWD 1 0" "RR_BN_RECOMPUTE_MASK 1 0" "RR_SPLIT_DGRAD 1 0" "RR_STREAM3_CONCAT 1 0" "RR_IMGGRAD_PERSIST 1 0" "RR_FUSED_POOL_BWD 1 0" "RR_BN_PAIR_FINALIZE 1 0" || exit 1
cat gpurun_out/ab_multi.txt
