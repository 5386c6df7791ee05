// swgrad.h -- internal interface of the row-streaming 3x3 weight gradient
// (swgrad.hip), called from rr_wgrad (wgrad.hip).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/roadrestore.h"

struct SWArgs {
  const char *dy;            // NHWC bf16 [n][h][w][cout]; a workgroup reads one 64-channel slice
  const char *x1, *x2;       // NHWC bf16 [n][h][w][c1], [n][h][w][c2] (concat input)
  int c1, c2;
  int cout;                  // dy channels (a multiple of 64)
  float *partial;            // [nwg_ps][cout][9][c1 + c2] partial dW slabs
  int n, h;                  // w is the template width
  int nwg_ps;                // workgroups per (dy slice, input slice) pair
  int nsteps;                // 128-pixel steps (n h w / 128)
  // input transform (swgrad_launch_pre): x1 is the pre-BN t1 of a
  // ResidualBlock's conv1; the kernel reads PReLU(t1 * pre_s + pre_b)
  const float *pre_s, *pre_b, *pre_alpha;
};

// nonzero when the descriptor is handled by the streaming kernel
int swgrad_ok(const rr_wgrad_desc *d);
// number of [64][9][c_in1 + c_in2] fp32 partial slabs the kernel writes
int swgrad_nsplit(const rr_wgrad_desc *d);
// launches the streaming kernel into ws (the caller reduces the slabs)
int swgrad_launch(const rr_wgrad_desc *d, const void *dy, const void *x1, const void *x2, void *ws,
                  hipStream_t st);
// the same with x1 = t1 and BN1 + PReLU applied to every landed input row
// ((s, b) of [c_in1] fp32, alpha [1]); single-source inputs only
int swgrad_launch_pre(const rr_wgrad_desc *d, const void *dy, const void *x1, const float *pre_s,
                      const float *pre_b, const float *pre_alpha, void *ws, hipStream_t st);
