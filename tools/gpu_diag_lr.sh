for e in "X=1" "RR_FUSE_BNBWD=0" "RR_FUSED_FIRST_WGRAD=0" "RR_FUSED_POOL=0"; do
  echo "== $e"; env $e timeout -k 10 100 python tools/diag_lr.py 2>&1 | grep -v amdgpu.ids | grep -E "step [0-5]|worst grad" || exit 1
done
