/*
 * roadrestore.h -- C ABI of the MI355X (gfx950) hot path of the road-sign
 * restoration pipeline.
 *
 * The reference (LordTARN1SHED/Image-Restoration-for-Road-Sign-Recognition-in-
 * Autonomous-Driving) has no FFI: its hot path is torch.nn.Module.forward +
 * autograd dispatching ATen conv / BN / PReLU / pool / convT / cat kernels
 * (SURVEY.md §2.3, §8b).  Each entry point below replaces one of those ATen
 * calls as issued by the reference modules; the reference call site is cited
 * on every declaration.  The Python host side (roadrestore/, ctypes) binds
 * exactly these symbols -- see INTEGRATION.md.
 *
 * Conventions
 *  - Activations are NHWC (channels contiguous), dtype RR_F32 or RR_BF16.
 *    Model inputs/outputs at the module boundary are NCHW fp32.
 *  - All buffers are device pointers owned by the caller; the library never
 *    allocates device memory.  Scratch comes from a caller workspace whose size
 *    is reported by the matching *_workspace() query.
 *  - Every launcher is asynchronous on `stream` (a hipStream_t) and returns an
 *    rr_status: 0 ok, <0 error (bad descriptor, unsupported shape, launch
 *    failure).  No C++ exception crosses the ABI.
 */
#ifndef ROADRESTORE_H
#define ROADRESTORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *rr_stream;   /* hipStream_t */

enum rr_status {
  RR_OK = 0,
  RR_EINVAL = -1,        /* malformed descriptor / null pointer            */
  RR_EUNSUPPORTED = -2,  /* shape outside what the kernels implement       */
  RR_ELAUNCH = -3,       /* hipLaunchKernel / runtime error                */
  RR_EWORKSPACE = -4     /* workspace smaller than *_workspace() reported  */
};

enum rr_dtype { RR_F32 = 0, RR_BF16 = 1 };

/* implicit-GEMM geometry (how the activation operand is gathered) */
enum rr_igemm_mode {
  RR_CONV3X3 = 0,   /* 3x3, stride 1, pad 1: fwd conv and its dgrad        */
  RR_CONV1X1 = 1,   /* 1x1 conv, shortcut conv, Linear (h = w = 1)         */
  RR_CONVT_UP = 2,  /* ConvTranspose2d(k2,s2) fwd: GEMM + 2x2 pixel scatter */
  RR_CONVT_DOWN = 3 /* ConvTranspose2d(k2,s2) dgrad: gather 2x2 -> GEMM     */
};

enum rr_act { RR_ACT_NONE = 0, RR_ACT_RELU = 1, RR_ACT_PRELU = 2 };
/* act flags (rr_igemm_ex): res[p, c] (y's layout) added before the
 * activation; the 2x2 max-pool of the final output also written to y_pool
 * [n][h/2][w/2][c_out] (nn.MaxPool2d(2) after it, floor sizes); NOFULL: only
 * the pooled output (y1 not written) */
#define RR_ACT_RES 4
#define RR_ACT_POOL 8
#define RR_ACT_NOFULL 16

/*
 * Implicit-GEMM convolution: y[p, c] = sum_k W[c, k] * X[p, k] (+ epilogue).
 *   p runs over the n*h*w pixels of the GEMM's row grid, c over c_out
 *   GEMM columns (RR_CONVT_UP: c_out = 4*Cout, column = tap*Cout + co),
 *   k over taps x (c_in1 + c_in2) input channels (two NHWC sources = the
 *   reference's torch.cat((up, skip), 1) read in place, 07:112, 14:174).
 */
typedef struct {
  int32_t dtype;       /* rr_dtype of x1, x2, w, y                          */
  int32_t mode;        /* rr_igemm_mode                                     */
  int32_t n, h, w;     /* GEMM row grid (output pixels; convT_up: input px)  */
  int32_t c_in1;       /* channels of source 1 (the "up" half of a cat)      */
  int32_t c_in2;       /* channels of source 2 (skip half) or 0              */
  int32_t c_out;       /* GEMM columns                                       */
  int32_t out_split;   /* columns [0,out_split) -> y1, rest -> y2; 0 = all y1 */
  int32_t act;         /* rr_act applied after bias                          */
  int32_t accumulate;  /* 1: y = y_old + result (before act/mask)            */
  int32_t has_bias;    /* bias[c] (fp32) added                               */
  int32_t has_mask;    /* result *= (mask[p, c] > 0); mask has y's layout    */
  int32_t want_stats;  /* per-(row-block, column) partial sum / sum of squares */
  int32_t out_nchw;    /* y1 is fp32 NCHW [n][c_out][h][w] (model boundary:
                          the 64->3 final conv 07:96 / 14:149, and the image
                          grad of the perceptual slice's conv1_1, 14:196) */
} rr_igemm_desc;

/* packed weights: w[c_out][taps][c_in1+c_in2] in dtype (see rr_pack_*; a
 * bf16 3x3 conv the tap-reuse kernel takes also reads the tiles behind it). */
int rr_igemm(const rr_igemm_desc *d, const void *x1, const void *x2,
             const void *w, const float *bias, void *y1, void *y2,
             const void *mask, float *stats_partial, rr_stream stream);
/* rr_igemm with the inference epilogues of a residual block fused (eval mode,
 * BatchNorm folded into the conv, 17:84-86; ResidualBlock 14:96-115):
 *   act & 3 == RR_ACT_PRELU: y = PReLU_alpha(conv + bias), alpha[0] the
 *     single nn.PReLU() weight (conv_block[2]);
 *   act & RR_ACT_RES: res[p, c] (y1's layout) added before the activation --
 *     the identity shortcut's relu(conv2(a1) + x);
 *   act & RR_ACT_POOL (+ RR_ACT_NOFULL): the encoder's / VGG's 2x2 max-pool
 *     of the result (14:127-131, torchvision vgg16 features) to y_pool.
 * bf16 3x3 convs the tap-reuse kernel takes (rr_igemm_kernel_name reports
 * "conv3r_kernel<...>" for the descriptor); no split / accumulate / NCHW
 * output with these flags.  Other descriptors: RR_EUNSUPPORTED. */
int rr_igemm_ex(const rr_igemm_desc *d, const void *x1, const void *x2, const void *w,
                const float *bias, const float *alpha, const void *res, void *y1,
                void *y_pool, const void *mask, float *stats_partial, rr_stream stream);
/* conv (+ bias) + ReLU + MaxPool2d(2, 2) (floor) in one pass, the full-size
 * output never written: y_pool [n][h/2][w/2][c_out] and, when pool_idx is
 * not null, the first-max window index (0..3, rr_maxpool2_fwd's) for the
 * backward (rr_maxpool2_bwd_pooled).  The perceptual VGG slice's conv + ReLU
 * + MaxPool2d pairs (torchvision vgg16 features[2:5], [7:10], 14:189-196).
 * d->act must be RR_ACT_RELU; no split / accumulate / mask / statistics.
 * bf16 3x3: the row-streaming kernel (64 -> 64 channels, 64x64 / 32x32 maps;
 * needs pool_idx) or the tap-reuse conv; others RR_EUNSUPPORTED. */
int rr_igemm_pool(const rr_igemm_desc *d, const void *x1, const void *x2, const void *w,
                  const float *bias, void *y_pool, uint8_t *pool_idx, rr_stream stream);
/* the kernel rr_igemm_pool launches for *d, or "unsupported" */
const char *rr_igemm_pool_kernel_name(const rr_igemm_desc *d);
/* y = the 3x3 dgrad of dy (d: mode RR_CONV3X3, c_in1 = dy's channels, c_out =
 * y's; no bias / activation / statistics / mask / split / accumulate) + the
 * 1x1 dgrad of a second gradient dy_sc [n][h][w][c_sc] with w_sc, the rows of
 * y's channels in the 1x1 conv's dgrad pack ([c_out][c_sc], rr_pack_conv) --
 * one pass, fp32 sum of both, rounded once.  A ResidualBlock's input grad =
 * conv_block[0]'s dgrad + shortcut[0]'s dgrad (14:99-115; dec1's concat
 * halves).  bf16, 64 -> 64 channels, c_sc = 64, the row-streaming kernel's
 * maps (64x64 / 32x32); others RR_EUNSUPPORTED (the caller runs rr_igemm +
 * an accumulating 1x1 rr_igemm).  Replaces the two torch autograd dgrads of
 * nn.Conv2d at 14:99-113. */
int rr_igemm_dgrad_sc(const rr_igemm_desc *d, const void *dy, const void *w, const void *dy_sc,
                      const void *w_sc, int c_sc, void *y, rr_stream stream);
/* the kernel rr_igemm_dgrad_sc launches for (*d, c_sc), or "unsupported" */
const char *rr_igemm_dgrad_sc_kernel_name(const rr_igemm_desc *d, int c_sc);
/* A ResidualBlock's conv2 forward with BatchNorm1 + PReLU of its input folded
 * in (14:101-104, training): x1 = t1 (conv1's pre-BN output) and the conv
 * reads a1 = PReLU(t1 * pre_scale[c] + pre_shift[c]) with alpha pre_alpha[0] --
 * bitwise the bytes rr_affine_act(t1, pre_scale, pre_shift, alpha) would store,
 * applied to every input row as it lands in the row-streaming kernel's ring,
 * so a1 is never written.  d: the bias + BN-statistics forward (has_bias,
 * want_stats, no act / mask / split / accumulate / second source) on the
 * row-streaming kernel's 64 -> 64 whole-row maps (rr_igemm_pre_ok != 0);
 * others RR_EUNSUPPORTED (the caller runs rr_affine_act + rr_igemm).
 * Replaces bn1 + prelu + conv2 of conv_block at 14:99-105. */
int rr_igemm_pre_ok(const rr_igemm_desc *d);
int rr_igemm_pre(const rr_igemm_desc *d, const void *x1, const void *w, const float *bias,
                 const float *pre_scale, const float *pre_shift, const float *pre_alpha,
                 void *y1, float *stats_partial, rr_stream stream);
/* number of row blocks the partial stats buffer holds: [blocks][c_out][2] */
int rr_igemm_stat_blocks(const rr_igemm_desc *d);
/* The kernel rr_igemm (bnbwd = 0) or rr_igemm_bnbwd (bnbwd = 1) launches for
 * *d, e.g. "stream3_kernel<64>", "igemm3_halo_kernel<64,32>",
 * "igemm_kernel<bf16,128,128,m1>" (m = mode).  Static string, never NULL; no
 * launch, no device needed.  Used to name the roofline kernel and to assert
 * which schedule a test exercises. */
const char *rr_igemm_kernel_name(const rr_igemm_desc *d, int bnbwd);

/* conv dgrad fused with the backward reduce of the BatchNorm2d -> PReLU pair
 * that produced its input (ResidualBlock conv_block[1:3], 14:101-103):
 * the GEMM result is g = dL/d(PReLU out); the epilogue writes
 *   gm = g * (u > 0 ? 1 : alpha),  u = t * aff_s[c] + aff_b[c] (BN output)
 * to gm_out and the partials partial[rows][c_out][3] = {sum gm, sum gm*xhat, 0}
 * (xhat = (t - mean) * invstd) followed by partial_alpha[rows][c_out/64] of
 * sum(g * u * (u <= 0)), rows = rr_igemm_stat_blocks(d).  Replaces the
 * separate rr_bn_bwd_reduce pass (mask_kind 2) over dL/d(PReLU out).
 * d: no bias / split / mask / accumulate / stats / act, c_in2 = 0,
 * c_out % 64 == 0. */
size_t rr_igemm_bnbwd_workspace(const rr_igemm_desc *d);
int rr_igemm_bnbwd(const rr_igemm_desc *d, const void *dy, const void *w, const void *t,
                   const float *mean, const float *invstd, const float *aff_s,
                   const float *aff_b, const float *alpha, void *gm_out, float *partial,
                   rr_stream stream);

/*
 * Weight-gradient GEMM (split over pixels):
 *  RR_CONV3X3 / RR_CONV1X1:  dW[co][ci][ky][kx] = sum_p dy[p,co] x[p+tap,ci]
 *  RR_CONVT_UP:              dW[ci][co][ky][kx] = sum_p x[p,ci] dy[2p+tap,co]
 *  (nn.Conv2d / nn.ConvTranspose2d weight grads of the reference modules).
 *  dw is fp32 in torch's layout; accumulate adds into it.
 */
typedef struct {
  int32_t dtype;
  int32_t mode;        /* RR_CONV3X3, RR_CONV1X1 or RR_CONVT_UP              */
  int32_t n, h, w;     /* conv: output grid (= input grid); convT: input grid */
  int32_t c_in1, c_in2;/* x channels (two sources for a cat input)           */
  int32_t c_out;       /* dy channels                                        */
  int32_t accumulate;
} rr_wgrad_desc;

size_t rr_wgrad_workspace(const rr_wgrad_desc *d);
/* The weight-grad kernel rr_wgrad launches for *d ("swgrad_kernel<64>",
 * "wgrad3_halo_kernel<16>", "wgrad_kernel<bf16,128,64,m1>", ...); static string. */
const char *rr_wgrad_kernel_name(const rr_wgrad_desc *d);
int rr_wgrad(const rr_wgrad_desc *d, const void *dy, const void *x1,
             const void *x2, float *dw, void *ws, size_t ws_bytes,
             rr_stream stream);
/* rr_wgrad in its two launches: the weight-grad kernel writing the split
 * partials into ws, and the fixed-order reduce of ws into dw (same result as
 * rr_wgrad, bitwise).  The reduce may run on another stream once the partial
 * launch has completed there (the training step puts it beside the next
 * dgrad, off the critical path). */
int rr_wgrad_partial(const rr_wgrad_desc *d, const void *dy, const void *x1,
                     const void *x2, void *ws, size_t ws_bytes, rr_stream stream);
int rr_wgrad_reduce(const rr_wgrad_desc *d, const void *ws, size_t ws_bytes, float *dw,
                    rr_stream stream);
/* conv2's weight grad with BatchNorm1 + PReLU of its input folded in (the
 * backward of rr_igemm_pre): x1 = t1, the kernel reads PReLU(t1 * pre_scale +
 * pre_shift) as rr_igemm_pre does; partial launch + rr_wgrad_reduce, bitwise
 * rr_wgrad on the stored a1.  d: RR_CONV3X3, one source, no accumulate, the
 * row-streaming weight grad's maps (rr_wgrad_pre_ok != 0); others
 * RR_EUNSUPPORTED.  Replaces conv_block[3]'s weight grad at 14:99-105. */
int rr_wgrad_pre_ok(const rr_wgrad_desc *d);
int rr_wgrad_pre(const rr_wgrad_desc *d, const void *dy, const void *x1, const float *pre_scale,
                 const float *pre_shift, const float *pre_alpha, float *dw, void *ws,
                 size_t ws_bytes, rr_stream stream);

/* weight packing (fp32 torch layout -> compute layout/dtype) */
/* conv [co][ci][k][k] -> fwd [co][k*k][ci] and dgrad [ci][k*k flipped][co].
 * bf16 3x3 convs with c_in, c_out multiples of 32 also get, right after that
 * layout, the 1-KB weight tiles the tap-reuse conv reads (one contiguous run
 * per (32-channel chunk, tap column, tap row)): each pack buffer then holds
 * rr_pack_conv_elems() = 2 * c_out * 9 * c_in elements. */
long long rr_pack_conv_elems(int dtype, int c_out, int c_in, int k);
int rr_pack_conv(int dtype, int c_out, int c_in, int k, const float *w,
                 void *w_fwd, void *w_dgrad, rr_stream stream);
/* convT [ci][co][2][2] -> up [tap*co][ci] and down [ci][tap][co] */
/* every conv pack of a network in one launch (the per-step re-pack after the
 * optimizer step): jobs[count] in DEVICE memory, job j covering elements
 * [begin, next begin) of a virtual concatenation of the fp32 weights; total =
 * sum of c_out * c_in * k * k.  Same layouts (and tiles) as rr_pack_conv. */
typedef struct rr_pack_job {
  const float *w;      /* [c_out][c_in][k][k] fp32                         */
  void *w_fwd;         /* [c_out][k*k][c_in] or NULL                       */
  void *w_dgrad;       /* [c_in][flipped k*k][c_out] or NULL               */
  int32_t c_out, c_in, k, pad_;
  int64_t begin;       /* first element of this job                        */
} rr_pack_job;
int rr_pack_conv_batch(int dtype, int count, const rr_pack_job *jobs,
                       long long total, rr_stream stream);
int rr_pack_convT(int dtype, int c_in, int c_out, const float *w,
                  void *w_up, void *w_down, rr_stream stream);
/* replicate bias over the 4 taps of a convT: b4[tap*co] = b[co] */
int rr_bias_tile4(int c_out, const float *b, float *b4, rr_stream stream);

/*
 * BatchNorm2d (14:101-112; eps, momentum as given).  stats_partial is the
 * [blocks][C][2] output of rr_igemm(want_stats) over the PRE-BIAS accumulator;
 * bias is that conv's bias (may be NULL).  Writes scale/shift (the affine the
 * apply kernels use), save_mean / save_invstd (for backward) and updates the
 * running stats in place (unbiased var), like F.batch_norm(training=True).
 * momentum < 0: the cumulative moving average of nn.BatchNorm2d(momentum=None),
 * factor 1 / (num_batches_tracked + 1) read on the device (num_batches_tracked
 * required; no host synchronisation, graph-capturable).
 */
int rr_bn_finalize(int C, int blocks, long long count, const float *stats_partial,
                   const float *bias, const float *gamma, const float *beta,
                   float *running_mean, float *running_var, float momentum,
                   float eps, float *scale, float *shift, float *save_mean,
                   float *save_invstd, int64_t *num_batches_tracked, void *ws,
                   size_t ws_bytes, rr_stream stream);
/* rr_bn_finalize's arguments as one descriptor */
typedef struct rr_bn_finalize_desc {
  int32_t C, blocks;
  int64_t count;
  const float *part, *bias, *gamma, *beta;
  float *running_mean, *running_var;
  float momentum, eps;
  float *scale, *shift, *save_mean, *save_invstd;
  int64_t *num_batches_tracked;
} rr_bn_finalize_desc;
/* two rr_bn_finalize calls as ONE launch: the residual tail's BatchNorm and
 * the shortcut's (14:109-114), whose statistics are ready together.  Direct
 * path only (blocks <= 8192 for both): else RR_EUNSUPPORTED, nothing done. */
int rr_bn_finalize_pair(const rr_bn_finalize_desc *a, const rr_bn_finalize_desc *b,
                        rr_stream stream);
/* workspace of rr_bn_finalize: 0 for blocks <= 8192 (one workgroup per channel
 * sums the raw partials in place; ws may be NULL); above that the
 * [blocks][C][2] partials are first folded to <= 64 fp64 rows by a parallel
 * fixed-order column reduction in ws */
size_t rr_bn_finalize_workspace(int C, int blocks);
/* eval-mode BatchNorm folded into the conv that feeds it (inference,
 * 17:84-85): w_out[c][k] = w[c][k] * scale[c], b_out[c] = b[c] * scale[c] +
 * shift[c] (scale / shift from rr_bn_eval_affine; b may be NULL); fp32,
 * torch weight layout [co][kel] */
int rr_fold_conv_bn(int co, int kel, const float *w, const float *b, const float *scale,
                    const float *shift, float *w_out, float *b_out, rr_stream stream);
/* eval mode: scale/shift from running stats (17:64 model.eval()) */
int rr_bn_eval_affine(int C, const float *gamma, const float *beta,
                      const float *running_mean, const float *running_var,
                      float eps, float *scale, float *shift, rr_stream stream);

/*
 * Fused elementwise forward over NHWC [P][C]:
 *   u = x*scale[c] + shift[c];  u = prelu(u, alpha) if alpha != NULL
 *   if res != NULL: u += (res_scale ? res*res_scale[c]+res_shift[c] : res)
 *   if relu: u = max(u, 0)
 * (PReLU(BN(conv)) 14:101-103 and relu(BN(conv) + shortcut) 14:115.)
 */
int rr_affine_act(int dtype, long long P, int C, const void *x, const float *scale,
                  const float *shift, const float *alpha, const void *res,
                  const float *res_scale, const float *res_shift, int relu,
                  void *y, rr_stream stream);

/*
 * BatchNorm backward, reduction half.  Upstream grad g on the BN output side:
 *   mask_kind 0: gm = g
 *   mask_kind 1: gm = g * (aux > 0)                  (relu after the add, 14:115)
 *   mask_kind 2: u = aux*aff_s[c]+aff_b[c]; gm = g*(u>0 ? 1 : alpha)
 *                and alpha_grad partial += g*u*(u<=0)   (PReLU, 14:103)
 * For up to two BNs fed by the same gm (BN2 and the shortcut BN) it produces
 * per-row-block partials of sum(gm) and sum(gm * xhat_i), xhat_i = (t_i -
 * mean_i) * invstd_i.  partial layout [blocks][C][3] (+ alpha partial).
 */
typedef struct {
  int32_t dtype;
  int64_t P;
  int32_t C;
  int32_t mask_kind;    /* 0 none, 1 ReLU (aux = ReLU output), 2 PReLU (aux = t),
                           3 ReLU + MaxPool2d(2,2) backward: g + unpool(pool_dy, pool_idx)
                           before the mask (the encoder block output feeds both the
                           skip concat and the pool, 14:125-131),
                           4 / 5 as 1 / 3 with nbn = 2 (residual tail with a BN
                           shortcut, 14:107-115) but the ReLU mask recomputed from
                           t0, t1 as the forward computed the block output:
                           relu(t0*aff_s[c] + aff_b[c] + (t1*aff_s[C+c] + aff_b[C+c]));
                           aux unused, aff_s / aff_b are [2][C], no gm_out */
  int32_t nbn;          /* 1 or 2 */
  int32_t h, w;         /* mask_kind 3: the [P] rows are [n][h][w] pixels (h, w even) */
  const void *pool_dy;  /* mask_kind 3: [n][h/2][w/2][C] grad of the pooled output */
  const uint8_t *pool_idx; /* mask_kind 3: rr_maxpool2_fwd / rr_affine_act_pool index */
  int32_t eval;         /* 1: eval-mode BatchNorm (mean / invstd are the running
                           statistics, which do not depend on the batch): the
                           finalize drops the mean(gm) and mean(gm * xhat) terms,
                           so dt = gamma * invstd * gm, and writes the grad of
                           the conv bias feeding BN i, gamma_i * invstd_i * sum(gm),
                           to dbias_i (NULL: skipped) -- in training mode that
                           grad is exactly zero */
  float *dbias0, *dbias1;
} rr_bnbwd_desc;
/* residual tail (as rr_affine_act, without PReLU) over an [n][h][w][C] NHWC
 * activation fused with MaxPool2d(2, 2) (14:125-131): y, the pooled y_pool
 * [n][h/2][w/2][C] and the first-max window index idx (as rr_maxpool2_fwd,
 * on the stored values) */
int rr_affine_act_pool(int dtype, int n, int h, int w, int C, const void *x,
                       const float *scale, const float *shift, const void *res,
                       const float *res_scale, const float *res_shift, int relu,
                       void *y, void *y_pool, uint8_t *idx, rr_stream stream);
int rr_bn_bwd_blocks(const rr_bnbwd_desc *d);
int rr_bn_bwd_reduce(const rr_bnbwd_desc *d, const void *g, const void *aux,
                     const float *aff_s, const float *aff_b, const float *alpha,
                     const void *t0, const float *mean0, const float *invstd0,
                     const void *t1, const float *mean1, const float *invstd1,
                     float *partial, rr_stream stream);
/* rr_bn_bwd_reduce for one BN behind a ReLU-masked identity residual tail
 * (mask_kind 1, or 3 with the 2x2 max-pool backward; C % 8 == 0 and C / 8
 * divides 256) that also stores gm = the masked upstream grad, rounded to the
 * dtype -- the residual branch's input grad (ResidualBlock without a shortcut
 * conv, 14:110-115) -- and sums the stored values.  The apply then reads gm
 * alone (rr_bn_bwd_apply with mask_kind 0, g = gm) instead of the upstream
 * grad, the pooled grad, its window index and the block output again. */
int rr_bn_bwd_reduce_gm(const rr_bnbwd_desc *d, const void *g, const void *aux,
                        const void *t0, const float *mean0, const float *invstd0,
                        float *partial, void *gm_out, rr_stream stream);
/* finalize: dgamma/dbeta (fp32, written) and the per-channel coefficients */
int rr_bn_bwd_finalize(const rr_bnbwd_desc *d, const float *partial,
                       const float *gamma0, const float *invstd0,
                       const float *gamma1, const float *invstd1,
                       float *dgamma0, float *dbeta0, float *dgamma1, float *dbeta1,
                       float *dalpha, float *coef, rr_stream stream);
/* finalize from caller-provided row partials [rows][C][3] (e.g. the
 * rr_igemm_bnbwd epilogue), fp64 fixed-order reduce; nbn = 1.  arows /
 * apartial: the PReLU alpha partials (0 / NULL when none). */
size_t rr_bn_bwd_finalize_rows_workspace(int C, int rows);
int rr_bn_bwd_finalize_rows(const rr_bnbwd_desc *d, int rows, const float *partial, int arows,
                            const float *apartial, const float *gamma0, const float *invstd0,
                            float *dgamma0, float *dbeta0, float *dalpha, float *coef,
                            void *ws, size_t ws_bytes, rr_stream stream);
/* the final 1x1 conv's backward (dw, db as rr_conv_out_bwd; its input grad g
 * NOT stored) fused with the reduce of the residual-tail BN backward of the
 * block that produced its input x (ResUNet dec1 -> final, 14:99-115, 14:149):
 * bn_partial [rr_bn_bwd_blocks(d)][C][3] for rr_bn_bwd_finalize, gm = g
 * rounded to the activation dtype, masked by x > 0 (x = the block output).
 * d: mask_kind 4, nbn 2, P = n*h*w, C = 64 (t0 / t1: the block's two pre-BN
 * tensors, as rr_bn_bwd_reduce); cout = 3.  The apply is
 * rr_bn_bwd_apply_convout.  Replaces the autograd of nn.Conv2d(64, 3, 1) and
 * the reduce half of BatchNorm2d's backward at 14:149 / 14:104-115. */
size_t rr_conv_out_bwd_bnred_workspace(long long P, int cin, int cout);
int rr_conv_out_bwd_bnred(const rr_bnbwd_desc *d, int n, int h, int w, int cout, const float *dy,
                          const void *x, const float *wt, const void *t0, const float *mean0,
                          const float *invstd0, const void *t1, const float *mean1,
                          const float *invstd1, float *dw, float *db, float *bn_partial, void *ws,
                          size_t ws_bytes, rr_stream stream);
/* the apply of that BN backward (mask kind 4) with g recomputed from the
 * final conv's fp32 NCHW output grad dy [n][cout][h][w] and weights wt
 * [cout][C]: the 268 MB input grad is never written or read (cout = 3) */
int rr_bn_bwd_apply_convout(const rr_bnbwd_desc *d, int h, int w, const float *dy, const float *wt,
                            int cout, const float *aff_s, const float *aff_b, const void *t0,
                            const float *mean0, const float *invstd0, const void *t1,
                            const float *mean1, const float *invstd1, const float *coef,
                            void *dt0, void *dt1, rr_stream stream);
/* apply: dt_i = coef_a[c]*(gm - coef_b[c] - xhat_i*coef_c[c]); optional gm out */
int rr_bn_bwd_apply(const rr_bnbwd_desc *d, const void *g, const void *aux,
                    const float *aff_s, const float *aff_b, const float *alpha,
                    const void *t0, const float *mean0, const float *invstd0,
                    const void *t1, const float *mean1, const float *invstd1,
                    const float *coef, void *dt0, void *dt1, void *gm_out,
                    rr_stream stream);

/* per-channel column sums of an NHWC [P][C] tensor (bias grads), fp32 out */
int rr_channel_sum(int dtype, long long P, int C, const void *x, float *out,
                   int accumulate, void *ws, size_t ws_bytes, rr_stream stream);
size_t rr_channel_sum_workspace(long long P, int C);

/* per-block (sum, sum of squares) partials [blocks][C][2] of an NHWC [P][C]
   tensor, blocks = rr_bn_stats_blocks(P): the batch statistics of a
   standalone train-mode BatchNorm2d (torch.nn.BatchNorm2d.forward, the
   leaf-module path of 14:100-104 when called on its own), finalized by
   rr_bn_finalize with count = P */
int rr_bn_stats_blocks(long long P);
int rr_bn_stats(int dtype, long long P, int C, const void *x, float *partial, rr_stream stream);

/* MaxPool2d(2,2) floor mode (07:82, 14:125): y and 1-byte argmax (0..3) */
int rr_maxpool2_fwd(int dtype, int n, int h, int w, int C, const void *x,
                    void *y, uint8_t *idx, rr_stream stream);
/* gather-form backward: dx = (accumulate ? dx : 0) + scatter(dy by idx);
 * then dx *= (mask > 0) if mask (relu of the pooled activation, 07:81) */
int rr_maxpool2_bwd(int dtype, int n, int h, int w, int C, const void *dy,
                    const uint8_t *idx, void *dx, int accumulate,
                    const void *mask, rr_stream stream);
/* the same backward when the pool's input is a ReLU output (VGG16 features,
 * 14:189-196): the mask is taken from the POOLED forward output y_pool
 * [n][h/2][w/2][C] (the ReLU mask at a window's argmax is y_pool > 0; every
 * other element is 0 anyway), so the full-size activation need not be kept;
 * dx fully written (no accumulate).  Bitwise rr_maxpool2_bwd with mask =
 * the full-size ReLU output.  h, w even, C % 8 == 0. */
int rr_maxpool2_bwd_pooled(int dtype, int n, int h, int w, int C, const void *dy,
                           const uint8_t *idx, const void *y_pool, void *dx, rr_stream stream);

/* PNG encoding of restored uint8 HWC images (17:89-99: cv2.imwrite of the
 * BGR-swapped array, which stores the RGB pixels).  Host memory, no device:
 * 8-bit truecolour (c = 3) / greyscale (c = 1), zlib level 0..9, adaptive
 * per-row filter.  rr_png_encode: one image into out[cap]; returns the PNG
 * size (the bytes are written only when it fits) or a negative status.
 * rr_png_write_batch: n images of [h][w][c] into paths[i], on `threads` host
 * threads (<= 0: all hardware threads). */
long long rr_png_encode(int h, int w, int c, const uint8_t *hwc, int level, uint8_t *out,
                        long long cap);
int rr_png_write_batch(int n, int h, int w, int c, const uint8_t *hwc, const char *const *paths,
                       int level, int threads);

/* F.interpolate(x, size=(ho, wo)) mode 'nearest' on NHWC [n][hi][wi][C]
 * (ResUNet decoder skip alignment, 14:169-182; C % 4 == 0): ATen's source
 * index min(floor(o * (float)hi / ho), hi - 1) (identity / o >> 1 at equal /
 * doubled sizes), and its backward in deterministic gather form (dx of a
 * source pixel = the fixed-order sum of dy over the outputs it feeds). */
int rr_nearest_resize(int dtype, int n, int hi, int wi, int ho, int wo, int C,
                      const void *x, void *y, rr_stream stream);
int rr_nearest_resize_bwd(int dtype, int n, int hi, int wi, int ho, int wo, int C,
                          const void *dy, void *dx, rr_stream stream);

/* first layer: conv3x3 p1 from NCHW fp32 [n][cin][h][w] into NHWC dtype,
 * + bias, act: 0 none, 1 relu, 2 prelu(alpha)  (07:78 enc1.0, 14:122 enc1) */
int rr_conv_in_fwd(int dtype, int n, int h, int w, int cin, int cout,
                   const float *x, const float *wt, const float *b,
                   int act, const float *alpha, void *y, rr_stream stream);
/* MFMA form of the first conv: im2col of the NCHW fp32 image into an NHWC
 * [P][kpad] matrix (j = ci*9+ky*3+kx, column 9*cin = 1.0 carries the bias,
 * zero-padded to kpad, a multiple of the GEMM K step), and the matching
 * [cout][kpad] weight pack (bias in column 9*cin).  The conv is then
 * rr_igemm(RR_CONV1X1, c_in1 = kpad) and its weight+bias grad is
 * rr_wgrad(RR_CONV1X1) on the same im2col matrix. */
int rr_im2col3(int dtype, int n, int h, int w, int cin, int kpad, const float *x,
               void *col, rr_stream stream);
/* fused bf16 first conv (cin 3 -> cout 64; 07:78 enc1.0, 14:122 enc1,
 * VGG16 features[0] 14:189): im2col gathered in registers from the NCHW fp32
 * image, K = 27 taps + bias column padded to 32, one MFMA per 16x16 tile.
 * wpack32 = rr_pack_conv_in(RR_BF16, 64, 3, kpad = 32).  y_pre = conv + bias,
 * y_act = act(y_pre) with act 0 none / 1 relu / 2 prelu(alpha); NHWC bf16
 * [n][h][w][64], either may be NULL (y_act NULL requires act 0). */
int rr_conv_in_mfma(int n, int h, int w, const float *x, const void *wpack32, int act,
                    const float *alpha, void *y_pre, void *y_act, rr_stream stream);
int rr_pack_conv_in(int dtype, int cout, int cin, int kpad, const float *wt,
                    const float *b, void *out, rr_stream stream);
/* [cout][kpad] fp32 wgrad of that GEMM -> torch-layout dW [cout][cin][3][3], db */
int rr_unpack_conv_in_grad(int cout, int cin, int kpad, const float *g, float *dw,
                           float *db, rr_stream stream);
/* its weight/bias grads given dy (NHWC, pre-activation grad) */
int rr_conv_in_wgrad(int dtype, int n, int h, int w, int cin, int cout,
                     const float *x, const void *dy, float *dw, float *db,
                     void *ws, size_t ws_bytes, rr_stream stream);
size_t rr_conv_in_wgrad_workspace(int n, int h, int w, int cin, int cout);
/* input grad of that conv (VGG perceptual slice dgrad reaching the image) */
/* first-conv (3 -> 64) weight + bias grad fused with the backward of its
 * activation (act 1 ReLU 07:78, 2 PReLU 14:122-123), from the NCHW fp32
 * image, the bf16 NHWC grad of the activation output dy and the bf16
 * pre-activation t: dw [64][27], db [64], dalpha [1] (PReLU) written;
 * bf16 MFMA, deterministic */
size_t rr_conv_in_wgrad_act_workspace(int n, int h, int w);
int rr_conv_in_wgrad_act(int n, int h, int w, const float *x, const void *dy,
                         const void *t_pre, int act, const float *alpha,
                         float *dw, float *db, float *dalpha, void *workspace,
                         size_t workspace_bytes, rr_stream stream);
int rr_conv_in_dgrad(int dtype, int n, int h, int w, int cin, int cout,
                     const void *dy, const float *wt, float *dx, int accumulate,
                     rr_stream stream);
/* PReLU backward on an NHWC tensor (14:122 enc1's PReLU): dx = dy*(y_pre>0 ?
 * 1 : alpha); alpha_partial holds `blocks` per-workgroup partials and the
 * alpha gradient (their fixed-order sum) is written to *dalpha. */
int rr_prelu_bwd(int dtype, long long count, const void *dy, const void *y_pre,
                 const float *alpha, void *dx, float *alpha_partial, int blocks,
                 float *dalpha, rr_stream stream);

/* last layer: conv1x1 cin->cout (cout small) NHWC dtype -> NCHW fp32 (07:119) */
int rr_conv_out_fwd(int dtype, int n, int h, int w, int cin, int cout,
                    const void *x, const float *wt, const float *b, float *y,
                    rr_stream stream);
/* grads of the last layer: dx (NHWC dtype, optional mask by x>0),
 * dw / db (fp32, need workspace) from dy (NCHW fp32) */
int rr_conv_out_bwd(int dtype, int n, int h, int w, int cin, int cout,
                    const float *dy, const void *x, const float *wt,
                    void *dx, int mask_relu, float *dw, float *db, void *ws,
                    size_t ws_bytes, rr_stream stream);
size_t rr_conv_out_bwd_workspace(int n, int h, int w, int cin, int cout);

/* layout: NCHW fp32 <-> NHWC dtype */
int rr_nchw_to_nhwc(int dtype, int n, int c, int h, int w, const float *x,
                    void *y, rr_stream stream);
int rr_nhwc_to_nchw(int dtype, int n, int c, int h, int w, const void *x,
                    float *y, rr_stream stream);

/* mean losses (nn.L1Loss 14:219, nn.MSELoss 07:142, the perceptual
 * mean((F(x)-F(y))^2) 14:196): *out = (accumulate ? *out : 0) + scale *
 * mean(|a-b| or (a-b)^2), per-workgroup partials then a fixed-order sum. */
int rr_loss_fwd(int kind /*0 l1, 1 mse*/, int dtype, long long count,
                const void *a, const void *b, float *out_scalar, float scale,
                int accumulate, void *ws, size_t ws_bytes, rr_stream stream);
size_t rr_loss_workspace(long long count);
/* grad wrt a: g*scale/count * sign(a-b) (l1) or *2(a-b) (mse), g = *gscale_dev
 * (autograd's incoming grad, device scalar) or 1; optional grad wrt b;
 * mask_a_pos: the grad is zeroed where a <= 0 (a is a ReLU output: the
 * perceptual slice ends in relu3_3, 14:192). */
int rr_loss_bwd(int kind, int dtype, long long count, const void *a,
                const void *b, const float *gscale_dev, float scale, void *ga,
                void *gb, int accumulate, int mask_a_pos, rr_stream stream);

/* fused multi-tensor Adam/AdamW (14:222, 07:143) over a flat fp32 buffer */
int rr_adamw(long long count, float *param, const float *grad, float *m,
             float *v, float lr, float beta1, float beta2, float eps,
             float weight_decay, int decoupled, int step, rr_stream stream);
/* capturable AdamW/Adam (HIP graphs): *step_dev is incremented on the stream
 * first, then the update reads it; bias corrections as above, on device.  The
 * learning rate is *lr_dev (fp32, device): the LR schedule of 14:223, 248
 * (CosineAnnealingLR.step() per epoch) writes it between graph replays. */
int rr_adamw_dev(long long count, float *param, const float *grad, float *m, float *v,
                 const float *lr_dev, float beta1, float beta2, float eps,
                 float weight_decay, int decoupled, int64_t *step_dev, rr_stream stream);

/* inference post-processing (17:84-92): clamp(0,1)*255 -> uint8 HWC */
int rr_to_uint8_hwc(int n, int c, int h, int w, const float *x, uint8_t *out,
                    int bgr, rr_stream stream);
/* per-image PSNR between uint8 images (08:123, data_range 255), fp64 out */
int rr_psnr_u8(int n, long long per_image, const uint8_t *a, const uint8_t *b,
               double *out, rr_stream stream);
/* argmax over rows of [n][k] fp32 logits, first max on ties (18:47) */
int rr_argmax_rows(int n, int k, const float *logits, int64_t *out,
                   rr_stream stream);
/* AdaptiveAvgPool2d((oh,ow)) on NHWC -> NCHW-flatten order fp32-or-dtype
 * rows for the classifier (torch.flatten(x, 1) of NCHW) */
int rr_adaptive_avgpool_flatten(int dtype, int n, int h, int w, int C, int oh,
                                int ow, const void *x, void *y, rr_stream stream);

/* ---- image I/O either side of the networks ---- */

/* torchvision Resize((oh, ow)) of a PIL image == PIL Image.resize(BILINEAR)
 * (17_run_unified_inference.py:66, 18_test_unified_benchmark.py:28-32),
 * bit-exact, batched: in [n][h][w][c] uint8 (c <= 4).  out_kind 0: uint8
 * [n][oh][ow][c]; 1: fp32 [n][c][oh][ow] = ToTensor (x / 255) and, when
 * mean/std (host arrays of c floats) are given, Normalize (18:31). */
size_t rr_resize_workspace(int n, int h, int w, int c, int oh, int ow);
int rr_resize_bilinear_u8(int n, int h, int w, int c, int oh, int ow,
                          const uint8_t *in, int out_kind, const float *mean,
                          const float *std, void *out, void *workspace,
                          size_t workspace_bytes, rr_stream stream);

/* cv2.resize(img, (ow, oh)) with the default INTER_LINEAR, the clean image of
 * the 08 PSNR leg (08_run_inference.py:118-119): OpenCV's fixed-point
 * bilinear (resize.cpp resizeGeneric_, HResizeLinear / VResizeLinear; 11-bit
 * weights, the vertical pass as the x86 SIMD body VResizeLinearVec_32s8u
 * rounds, simd_lanes = its u8 vector width, 0 = 16), batched over [n][h][w][c]
 * uint8 (c <= 4) -> [n][oh][ow][c]; same size = copy.  Parity vs cv2 itself
 * is unpinned (cv2 is not installed where this was built). */
int rr_cv_resize_linear_u8(int n, int h, int w, int c, int oh, int ow,
                           const uint8_t *in, uint8_t *out, int simd_lanes,
                           rr_stream stream);

/* skimage structural_similarity(a, b, data_range=255, channel_axis=2)
 * (08_run_inference.py:125) per image of [n][h][w][c] uint8, fp64 out[n] */
size_t rr_ssim_workspace(int n, int c);
int rr_ssim_u8(int n, int h, int w, int c, const uint8_t *a, const uint8_t *b,
               double *out, void *workspace, size_t workspace_bytes,
               rr_stream stream);

/* distortion generator: apply_random_distortions 14:31-64 (mode 0: fog ->
 * noise -> motion blur) and apply_compound_distortion 16:14-37 (mode 1:
 * blur -> fog -> noise), per image parameters (drawn by the caller as the
 * reference draws them).  fog: x * fog_mul + fog_add in fp32 (fog_mul =
 * f32(t), fog_add = f32(A (1 - t))); noise: + N(0, sigma) in fp64, from
 * `noise` ([n][h][w][c] fp64) when given, else Philox4x32-10(seed); blur:
 * cv2.filter2D with the ksize x ksize taps of `taps` ([n][KMAX][KMAX]
 * fp32, rr_motion_blur_kernel), BORDER_REFLECT_101. */
#define RR_DISTORT_KMAX 15
enum { RR_DISTORT_FOG = 1, RR_DISTORT_NOISE = 2, RR_DISTORT_BLUR = 4 };
typedef struct rr_distort_param {
  double sigma;       /* noise standard deviation (var ** 0.5)            */
  float fog_mul;      /* f32(t)                                           */
  float fog_add;      /* f32(A * (1 - t))                                 */
  int32_t flags;      /* RR_DISTORT_* bits                                */
  int32_t ksize;      /* motion-blur degree (kernel side), <= KMAX        */
} rr_distort_param;
size_t rr_distort_workspace(int n, int h, int w, int c);
int rr_distort_u8(int n, int h, int w, int c, int mode, const uint8_t *in,
                  uint8_t *out, const rr_distort_param *params,
                  const float *taps, const double *noise,
                  unsigned long long seed, void *workspace,
                  size_t workspace_bytes, rr_stream stream);
/* host: the motion-blur kernel of 14:55-59 / 16:20-21 (cv2
 * getRotationMatrix2D + warpAffine of np.diag(np.ones(k)), / k, as fp32)
 * into taps[KMAX][KMAX] (row-major, zero outside k x k) */
int rr_motion_blur_kernel(int k, int angle, float *taps);

/* The whole apply_random_distortions (14:31-64) of a batch on device, graph-
 * capturable: the per-image draws (the reference's distributions: fog / noise
 * / blur each with p 0.5, intensity U(0.3, 0.7) x U(0.8, 1.2), var U(0.01,
 * 0.03), degree randint(5, 15), angle randint(0, 360)) come from
 * Philox4x32-10 keyed by (seed, *step), image index as counter; *step (device
 * int64) advances by one per call; the noise field uses a per-step Philox
 * seed.  `table` is the device copy of rr_motion_blur_table (all 11 x 361
 * blur kernels).  Then the same fog -> noise -> blur arithmetic as
 * rr_distort_u8 mode 0.  Replaces the host-side draws of the reference's
 * DataLoader workers (14:72-84, 213). */
size_t rr_motion_blur_table_floats(void);
int rr_motion_blur_table(float *table_host);
size_t rr_distort_random_workspace(int n, int h, int w, int c);
int rr_distort_random_u8(int n, int h, int w, int c, const uint8_t *in, uint8_t *out,
                         unsigned long long seed, long long *step_dev,
                         const float *table_dev, void *workspace, size_t workspace_bytes,
                         rr_stream stream);
/* byte offsets, inside that workspace, of the last call's draws (tests):
 * rr_distort_param[n], int32 table index[n], uint64 noise seed */
int rr_distort_random_draws(int n, int h, int w, int c, const void *workspace,
                            size_t *params_off, size_t *index_off, size_t *seed_off);

/* running loss on device: acc[0] += x[0] (fp64), count[0] += 1 -- the
 * reference's per-step `running_loss += loss.item()` (14:246) without a host
 * sync; read acc / count once per epoch */
int rr_scalar_accumulate(const float *x, double *acc, int64_t *count, rr_stream stream);

/* async memset of a device buffer (zero_grad of the flat buffers) */
int rr_zero(void *p, size_t bytes, rr_stream stream);

/* library version string */
const char *rr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ROADRESTORE_H */
