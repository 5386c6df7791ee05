#!/bin/bash
# per-stage vs fixed cost of the conv GEMM (diagnostic knobs of csrc/igemm.hip)
for d in 0 1 2 3; do
  echo "== RR_IGEMM_DBG=$d"
  RR_IGEMM_DBG=$d REPS=10 python tools/bench_gemm.py 2>&1 | grep -E "res1|dec1|bott.512|res3.c2" | cut -c1-80
done
