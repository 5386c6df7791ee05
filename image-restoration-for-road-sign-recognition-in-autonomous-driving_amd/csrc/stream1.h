// stream1.h -- internal interface of the wave-streaming 1x1 / convT GEMM
// (stream1.hip), called from rr_igemm (igemm.hip).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/roadrestore.h"

struct S1Args {
  const char *x1, *x2;       // NHWC bf16 sources (x2: second half of a concat input)
  const char *wt;            // packed bf16 weights [c_out][K] (the rr_igemm pack)
  const float *bias;         // per GEMM column or null
  char *y1, *y2;             // outputs (y2: columns >= split)
  const char *mask;          // relu-backward mask (y1 layout) or null
  float *stats;              // [G][c_out][2] pre-bias partial sums or null
  int mode, P, h, w, hw, lw, lhw;
  FastDiv fd_hw, fd_w;       // coarse pixel -> (image, row, column) for any h, w (convT up / down)
  int c1, c2, cout, cout_t, split, K, G, flags;
  int ksrc[16], kch[16], ktap[16];   // per 32-deep k fragment: source, channel, fine-grid tap offset
};

struct S1Plan {
  int mc, kb, nslice, G, key;
};

// workgroups per column slice (= rows of the stats partial slab) when the
// streaming kernel takes *d, else 0
int stream1_plan(const rr_igemm_desc *d, S1Plan *pl);
int stream1_launch(const rr_igemm_desc *d, const S1Plan &pl, S1Args a, hipStream_t st);
const char *stream1_name(const S1Plan &pl);
