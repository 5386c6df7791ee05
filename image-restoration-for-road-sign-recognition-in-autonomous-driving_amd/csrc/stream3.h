// stream3.h -- internal interface of the row-streaming 3x3 conv (stream3.hip),
// called from rr_igemm / rr_igemm_bnbwd (igemm.hip).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/roadrestore.h"

struct S3Args {
  const char *x;             // NHWC bf16 input [n][h][w][64]
  const char *x2;            // second 64-channel source of a concat input (two passes) or null
  const char *wt;            // packed bf16 weights [64][9][wld] (fwd or dgrad pack)
  int wld, woff;             // packed row length (c_in) and the pass's channel offset
  const float *bias;         // [64] or null
  char *y;                   // NHWC bf16 output [n][h][w][64]
  const char *mask;          // relu-backward mask (NHWC bf16) or null
  float *stats;              // [nwg][64][2] pre-bias partial sums or null
  int n, h, w;               // w: the image width (the template width, or a multiple: column strips)
  int act, accumulate;
  // BN -> PReLU backward epilogue (rr_igemm_bnbwd), bt != null selects it
  const char *bt;
  const float *bmean, *binv, *baff_s, *baff_b, *balpha;
  float *bpart, *bapart;     // [nwg][64][3], [nwg]
  // pool epilogue (stream3_launch_pool): 2x2 max-pool of the ReLU output and
  // its first-max window index, [n][h/2][w/2][64] (no full-size output)
  char *ypool;
  uint8_t *pidx;
  // 1x1 second source (stream3_launch_sc): NHWC bf16 [n][h][w][64] and its
  // weights [64 out][64] (rows of the 1x1 dgrad pack)
  const char *xsc, *wsc;
  // eval epilogues (stream3_launch_ex): PReLU alpha [1], identity residual NHWC bf16
  const float *alpha;
  const char *res;
  // input transform (stream3_launch_pre): x is the pre-BN t1, the conv reads
  // PReLU(t1 * pre_s + pre_b) ([64] fp32 each, pre_alpha [1])
  const float *pre_s, *pre_b, *pre_alpha;
};

// 0 when the descriptor is not handled by the streaming kernel, else the
// number of workgroups (= rows of the stats / bnbwd partial slabs); bnbwd:
// the rr_igemm_bnbwd epilogue.  Eligibility does not depend on the epilogue
// beyond the supported flag sets, so the partial-row count a caller sizes
// from the plain descriptor matches the launch.
int stream3_blocks(const rr_igemm_desc *d, int bnbwd);
// 1 when the streaming kernel walks *d in column strips (maps wider than 64):
// only the plain / bias / eval flag sets have strip instances (no statistics,
// operands, BN backward, 1x1 second source or pool window index)
int stream3_strips(const rr_igemm_desc *d);
// launch; returns an RR_* status
int stream3_launch(const rr_igemm_desc *d, const S3Args &a, int bnbwd, hipStream_t st);
// conv (+ bias) + ReLU + MaxPool2d(2, 2) with the window index (a.ypool,
// a.pidx; a.y unused); RR_EUNSUPPORTED when the streaming kernel does not
// take the descriptor
int stream3_launch_pool(const rr_igemm_desc *d, const S3Args &a, hipStream_t st);
// the plain 64 -> 64 dgrad plus a 1x1 dgrad of a.xsc with a.wsc into the same
// accumulators (rr_igemm_dgrad_sc); RR_EUNSUPPORTED when not taken
int stream3_launch_sc(const rr_igemm_desc *d, const S3Args &a, hipStream_t st);
// the BN-folded eval epilogues of rr_igemm_ex (d->act: PReLU, or ReLU with the
// identity residual and / or the 2x2 max-pool, no window index) on the
// streaming kernel: stream3_ex_ok() != 0 when it takes *d
int stream3_ex_ok(const rr_igemm_desc *d);
int stream3_launch_ex(const rr_igemm_desc *d, const S3Args &a, hipStream_t st);
// the bias + BN-statistics forward of conv2 with BN1 + PReLU applied to the
// landed input rows (a.pre_*): RR_EUNSUPPORTED unless the streaming kernel
// takes *d with whole rows and exactly that flag set
int stream3_launch_pre(const rr_igemm_desc *d, const S3Args &a, hipStream_t st);
// "stream3_kernel<64>" / "<32>" (whole rows) or "<s64>" / "<s32>" (column
// strips) + the suffix
const char *stream3_name(const rr_igemm_desc *d, const char *suffix);
