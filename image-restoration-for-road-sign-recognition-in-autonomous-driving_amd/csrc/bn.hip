// bn.hip -- BatchNorm2d / PReLU / residual elementwise kernels (NHWC, gfx950).
//
// Replaces the ATen kernels behind the reference's ResidualBlock
// (14_train_unified_advanced.py:96-115):
//   nn.BatchNorm2d train fwd (batch stats, running-stat update) / eval fwd /
//   backward, nn.PReLU fwd / bwd (single alpha), the residual add + ReLU, and
//   bias-gradient column sums.
// All of these are HBM-bound: one pass over [P][C] each, 16-B per lane
// accesses for fp32 (4 channels) and 8-B for bf16, per-channel reductions
// done as per-workgroup partials followed by a fixed-order finalize
// (deterministic, no float atomics).
#include "common.h"

// grid cap of the 8-channel grid-stride elementwise kernels (BN1 + PReLU
// apply, BN-backward apply): one resident round of 256-thread workgroups, so
// each workgroup's per-channel coefficient setup is paid once per ~16 rows.
// Graph-step A/B (profiles/r6zk_abstep_ew_grid.txt, r6zl_*): 2048 vs 4096
// +0.1-1.0 % in 5 of 6 pairs; 16384 -1 %, one row per thread -5 %.
#define RR_EW_GRID 2048

namespace {

// ---------------------------------------------------------------------------
// finalize of the conv-epilogue statistics -> scale / shift / running stats
// partial [blocks][C][2] of the pre-bias accumulator.
// 256 threads = 16 channels x 16 block-slices; double accumulation.
// BN statistics finalize straight from the raw fp32 per-tile partials
// [rows][C][2] (no column-reduce launch): one workgroup per channel, 256 row
// lanes in a fixed order + an LDS tree, then the same per-channel math as
// bn_finalize_kernel
struct BnFin {
  int C, rows;
  double count;
  const float *part, *bias, *gamma, *beta;
  float *rmean, *rvar;
  float momentum, eps;
  float *scale, *shift, *smean, *sinv;
  int64_t *nbt;
};

__device__ __forceinline__ void bn_finalize_direct_channel(const BnFin &a, int c);

__global__ __launch_bounds__(256) void bn_finalize_direct_kernel(
    int C, int rows, double count, const float *__restrict__ part, const float *bias,
    const float *gamma, const float *beta, float *rmean, float *rvar, float momentum, float eps,
    float *scale, float *shift, float *smean, float *sinv, int64_t *nbt) {
  const BnFin a{C, rows, count, part, bias, gamma, beta, rmean, rvar, momentum, eps, scale, shift,
                smean, sinv, nbt};
  bn_finalize_direct_channel(a, blockIdx.x);
}

// two BatchNorms finalized by one launch (the residual tail's BN and the
// shortcut BN, whose statistics are ready together): workgroups [0, A.C)
// take A's channels, the rest B's
__global__ __launch_bounds__(256) void bn_finalize_direct2_kernel(BnFin A, BnFin B) {
  if ((int)blockIdx.x < A.C) bn_finalize_direct_channel(A, blockIdx.x);
  else bn_finalize_direct_channel(B, blockIdx.x - A.C);
}

__device__ __forceinline__ void bn_finalize_direct_channel(const BnFin &a, int c) {
  const int C = a.C, rows = a.rows;
  const double count = a.count;
  const float *__restrict__ part = a.part;
  const float *bias = a.bias, *gamma = a.gamma, *beta = a.beta;
  float *rmean = a.rmean, *rvar = a.rvar, *scale = a.scale, *shift = a.shift, *smean = a.smean,
        *sinv = a.sinv;
  // momentum < 0: cumulative moving average (nn.BatchNorm2d(momentum=None)),
  // factor 1 / (num_batches_tracked + 1) read on the device; the count is then
  // incremented by a separate launch after this one (bn_nbt_inc_kernel)
  const bool cum = a.momentum < 0.f;
  const float eps = a.eps;
  __shared__ double red[2][256];
  const int t = threadIdx.x;
  if (a.nbt && !cum && c == 0 && t == 0) a.nbt[0] += 1;
  double s[2] = {0.0, 0.0};
  rr_fixed_sum<2>(part + ((long long)t * C + c) * 2, 256LL * C * 2, rr_trips(t, rows, 256), s);
  double s1 = s[0], s2 = s[1];
  red[0][t] = s1;
  red[1][t] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) { red[0][t] += red[0][t + o]; red[1][t] += red[1][t + o]; }
    __syncthreads();
  }
  if (t == 0) {
    s1 = red[0][0];
    s2 = red[1][0];
    const double mean_acc = s1 / count;
    double var = s2 / count - mean_acc * mean_acc;
    if (var < 0) var = 0;
    const double mean = mean_acc + (bias ? (double)bias[c] : 0.0);
    const double inv = 1.0 / sqrt(var + (double)eps);
    const double g = gamma ? (double)gamma[c] : 1.0;
    const double bt = beta ? (double)beta[c] : 0.0;
    scale[c] = (float)(g * inv);
    shift[c] = (float)(bt - mean * g * inv);
    if (smean) smean[c] = (float)mean;
    if (sinv) sinv[c] = (float)inv;
    const double momentum = cum ? 1.0 / (double)(a.nbt[0] + 1) : (double)a.momentum;
    if (rmean) rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    if (rvar) {
      const double unb = count > 1 ? var * count / (count - 1) : var;
      rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
    }
  }
}

__global__ void bn_nbt_inc_kernel(int64_t *nbt) { nbt[0] += 1; }

__global__ void bn_finalize_kernel(int C, int blocks, double count, const double *__restrict__ part,
                                   const float *bias, const float *gamma, const float *beta,
                                   float *rmean, float *rvar, float momentum, float eps,
                                   float *scale, float *shift, float *smean, float *sinv,
                                   int64_t *nbt) {
  __shared__ double red[2][16][17];
  const bool cum = momentum < 0.f;                  // as in bn_finalize_direct_channel
  if (nbt && !cum && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double s[2] = {0.0, 0.0};
  if (c < C) rr_fixed_sum<2>(part + ((long long)sl * C + c) * 2, 16LL * C * 2, rr_trips(sl, blocks, 16), s);
  double s1 = s[0], s2 = s[1];
  red[0][sl][cl] = s1;
  red[1][sl][cl] = s2;
  __syncthreads();
  if (sl == 0 && c < C) {
    for (int k = 1; k < 16; ++k) { s1 += red[0][k][cl]; s2 += red[1][k][cl]; }
    const double mean_acc = s1 / count;
    double var = s2 / count - mean_acc * mean_acc;
    if (var < 0) var = 0;
    const double mean = mean_acc + (bias ? (double)bias[c] : 0.0);
    const double inv = 1.0 / sqrt(var + (double)eps);
    const double g = gamma ? (double)gamma[c] : 1.0;
    const double bt = beta ? (double)beta[c] : 0.0;
    scale[c] = (float)(g * inv);
    shift[c] = (float)(bt - mean * g * inv);
    if (smean) smean[c] = (float)mean;
    if (sinv) sinv[c] = (float)inv;
    const double mom = cum ? 1.0 / (double)(nbt[0] + 1) : (double)momentum;
    if (rmean) rmean[c] = (float)((1.0 - mom) * rmean[c] + mom * mean);
    if (rvar) {
      const double unb = count > 1 ? var * count / (count - 1) : var;
      rvar[c] = (float)((1.0 - mom) * rvar[c] + mom * unb);
    }
  }
}

__global__ void bn_eval_kernel(int C, const float *gamma, const float *beta, const float *rm,
                               const float *rv, float eps, float *scale, float *shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = 1.0f / sqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  scale[c] = g * inv;
  shift[c] = b - rm[c] * g * inv;
}

// ---------------------------------------------------------------------------
template <typename T>
__global__ void affine_act_kernel(long long P, int C, const T *__restrict__ x,
                                  const float *__restrict__ scale, const float *__restrict__ shift,
                                  const float *alpha, const T *__restrict__ res,
                                  const float *__restrict__ rs, const float *__restrict__ rb,
                                  int relu, T *__restrict__ y) {
  const long long n4 = P * C / 4;
  const float al = alpha ? alpha[0] : 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    const long long e = i * 4;
    const int c = (int)(e % C);
    f32x4 v = load4<T>(x + e);
    const f32x4 s = *reinterpret_cast<const f32x4 *>(scale + c);
    const f32x4 b = *reinterpret_cast<const f32x4 *>(shift + c);
    v = v * s + b;
    if (alpha) {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = v[k] > 0.f ? v[k] : al * v[k];
    }
    if (res) {
      f32x4 r = load4<T>(res + e);
      if (rs) r = r * *reinterpret_cast<const f32x4 *>(rs + c) + *reinterpret_cast<const f32x4 *>(rb + c);
      v += r;
    }
    if (relu) {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = fmaxf(v[k], 0.f);
    }
    store4<T>(y + e, v);
  }
}

// 8-channel form of affine_act_kernel (C % 8 == 0, C / 8 divides 256): the
// thread's channel group is fixed over the grid-stride walk, so scale / shift
// live in registers and every access is a 16-B vector
template <typename T>
__global__ void affine_act8_kernel(long long P, int C, const T *__restrict__ x,
                                   const float *__restrict__ scale, const float *__restrict__ shift,
                                   const float *alpha, const T *__restrict__ res,
                                   const float *__restrict__ rs, const float *__restrict__ rb,
                                   int relu, T *__restrict__ y) {
  const int G = C / 8;
  const int c = (threadIdx.x % G) * 8;
  const f32x4 s0 = *reinterpret_cast<const f32x4 *>(scale + c), s1 = *reinterpret_cast<const f32x4 *>(scale + c + 4);
  const f32x4 b0 = *reinterpret_cast<const f32x4 *>(shift + c), b1 = *reinterpret_cast<const f32x4 *>(shift + c + 4);
  f32x4 r0s = {1.f, 1.f, 1.f, 1.f}, r1s = r0s, r0b = {0.f, 0.f, 0.f, 0.f}, r1b = r0b;
  if (rs) {
    r0s = *reinterpret_cast<const f32x4 *>(rs + c); r1s = *reinterpret_cast<const f32x4 *>(rs + c + 4);
    r0b = *reinterpret_cast<const f32x4 *>(rb + c); r1b = *reinterpret_cast<const f32x4 *>(rb + c + 4);
  }
  const float al = alpha ? alpha[0] : 0.f;
  const long long stride = ((long long)gridDim.x * blockDim.x) / G;
  for (long long r = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / G; r < P; r += stride) {
    const long long e = r * C + c;
    f32x4 v0, v1;
    load8<T>(x + e, v0, v1);
    v0 = v0 * s0 + b0;
    v1 = v1 * s1 + b1;
    if (alpha) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v0[k] = v0[k] > 0.f ? v0[k] : al * v0[k];
        v1[k] = v1[k] > 0.f ? v1[k] : al * v1[k];
      }
    }
    if (res) {
      f32x4 q0, q1;
      load8<T>(res + e, q0, q1);
      if (rs) { q0 = q0 * r0s + r0b; q1 = q1 * r1s + r1b; }
      v0 += q0;
      v1 += q1;
    }
    if (relu) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { v0[k] = fmaxf(v0[k], 0.f); v1[k] = fmaxf(v1[k], 0.f); }
    }
    store8<T>(y + e, v0, v1);
  }
}

// residual tail + MaxPool2d(2, 2) in one pass (14:114-115 then 14:125-131):
// y = relu(x * scale + shift + res * rs + rb) for the 4 pixels of a pooling
// window (8 channels per thread), and the window max / first-max index of
// the STORED (dtype-rounded) values -- exactly what maxpool2_fwd would read
template <typename T>
__global__ void affine_act_pool_kernel(int n, int h, int w, int C, const T *__restrict__ x,
                                       const float *__restrict__ scale, const float *__restrict__ shift,
                                       const T *__restrict__ res, const float *__restrict__ rs,
                                       const float *__restrict__ rb, int relu, T *__restrict__ y,
                                       T *__restrict__ yp, uint8_t *__restrict__ idx) {
  const int ho = h / 2, wo = w / 2, G = C / 8;
  const long long total = (long long)n * ho * wo * G;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int gq = (int)(i % G);
    const long long op = i / G;
    const int ox = (int)(op % wo);
    const long long tq = op / wo;
    const int oy = (int)(tq % ho);
    const int nn = (int)(tq / ho);
    const int c = gq * 8;
    const f32x4 s0 = *reinterpret_cast<const f32x4 *>(scale + c), s1 = *reinterpret_cast<const f32x4 *>(scale + c + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4 *>(shift + c), b1 = *reinterpret_cast<const f32x4 *>(shift + c + 4);
    f32x4 r0s = {1.f, 1.f, 1.f, 1.f}, r1s = r0s, r0b = {0.f, 0.f, 0.f, 0.f}, r1b = r0b;
    if (rs) {
      r0s = *reinterpret_cast<const f32x4 *>(rs + c); r1s = *reinterpret_cast<const f32x4 *>(rs + c + 4);
      r0b = *reinterpret_cast<const f32x4 *>(rb + c); r1b = *reinterpret_cast<const f32x4 *>(rb + c + 4);
    }
    float m[8];
    uint8_t id[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long long e = (((long long)nn * h + 2 * oy + (k >> 1)) * w + 2 * ox + (k & 1)) * C + c;
      f32x4 v0, v1, q0, q1;
      load8<T>(x + e, v0, v1);
      v0 = v0 * s0 + b0;
      v1 = v1 * s1 + b1;
      if (res) {
        load8<T>(res + e, q0, q1);
        if (rs) { q0 = q0 * r0s + r0b; q1 = q1 * r1s + r1b; }
        v0 += q0;
        v1 += q1;
      }
      if (relu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { v0[j] = fmaxf(v0[j], 0.f); v1[j] = fmaxf(v1[j], 0.f); }
      }
      store8<T>(y + e, v0, v1);
      // compare the stored values: round to T and back
      T rt[8];
      const float vv[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Elt<T>::store(rt, j, vv[j]);
        const float sv = Elt<T>::load(rt, j);
        if (k == 0) { m[j] = sv; id[j] = 0; }
        else {
          // branch-free first max (pool4_first_max's form: compares + selects)
          const bool t = !(sv <= m[j]) & (m[j] == m[j]);
          m[j] = t ? sv : m[j];
          id[j] = t ? (uint8_t)k : id[j];
        }
      }
    }
    store8<T>(yp + op * C + c, f32x4{m[0], m[1], m[2], m[3]}, f32x4{m[4], m[5], m[6], m[7]});
    *reinterpret_cast<uint2 *>(idx + op * C + c) =
        uint2{(uint32_t)id[0] | ((uint32_t)id[1] << 8) | ((uint32_t)id[2] << 16) | ((uint32_t)id[3] << 24),
              (uint32_t)id[4] | ((uint32_t)id[5] << 8) | ((uint32_t)id[6] << 16) | ((uint32_t)id[7] << 24)};
  }
}

// ---------------------------------------------------------------------------
// BN backward
struct BnBwd {
  long long P;
  int C, mask_kind, nbn;
  int h, w;                         // mask_kind 3: pixel grid of the rows
  const void *pdy;                  // mask_kind 3: pooled grad [n][h/2][w/2][C]
  const uint8_t *pidx;              // mask_kind 3: window index of the max
  const void *g, *aux;
  const float *aff_s, *aff_b, *alpha;
  const void *t0, *t1;
  const float *mean0, *inv0, *mean1, *inv1;
  // rr_bn_bwd_apply_convout: g = the final 1x1 conv's input grad, recomputed
  // from its fp32 NCHW output grad cody [n][3][h][w] and weights cow [3][C]
  const float *cody, *cow;
};

template <typename T>
__device__ __forceinline__ f32x4 bwd_gm(const BnBwd &a, long long e, int c, f32x4 &ag) {
  f32x4 g = load4<T>((const T *)a.g + e);
  ag = f32x4{0.f, 0.f, 0.f, 0.f};
  if (a.mask_kind == 1) {
    const f32x4 m = load4<T>((const T *)a.aux + e);
#pragma unroll
    for (int k = 0; k < 4; ++k) g[k] = m[k] > 0.f ? g[k] : 0.f;
  } else if (a.mask_kind == 2) {
    const f32x4 t = load4<T>((const T *)a.aux + e);
    const f32x4 u = t * *reinterpret_cast<const f32x4 *>(a.aff_s + c) +
                    *reinterpret_cast<const f32x4 *>(a.aff_b + c);
    const float al = a.alpha[0];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ag[k] = u[k] > 0.f ? 0.f : g[k] * u[k];
      g[k] = u[k] > 0.f ? g[k] : al * g[k];
    }
  }
  return g;
}

// ---- 8-channel forms (C % 8 == 0, C / 8 divides 256): a thread's channel
// group is fixed for the whole grid-stride walk, so the per-channel
// coefficients live in registers and every access is a 16-B vector.
//
// MASK 4 / 5 (nbn = 2, the residual tail with a BN shortcut): as 1 / 3, but
// the ReLU mask is recomputed from the two pre-BN tensors the kernel reads
// anyway, with the forward's own expression (affine_act8_kernel /
// affine_act_pool_kernel: v = t0*s0 + b0; q = t1*s1 + b1; v += q; relu), so
// the block output is not read: out > 0 <=> v > 0.  s8/b8 hold BN0's forward
// affine, sB/bB BN1's; tA/tB are the row's t0/t1 values.
template <typename T, int MASK, bool GIN = false>
__device__ __forceinline__ void bwd_gm8(const BnBwd &a, long long e, const float *s8,
                                        const float *b8, float al, float *g, float &ag,
                                        const float *tA = nullptr, const float *tB = nullptr,
                                        const float *sB = nullptr, const float *bB = nullptr) {
  if constexpr (!GIN) {                 // (GIN: g already holds the upstream grad)
    f32x4 g0, g1;
    load8<T>((const T *)a.g + e, g0, g1);
    g[0] = g0[0]; g[1] = g0[1]; g[2] = g0[2]; g[3] = g0[3];
    g[4] = g1[0]; g[5] = g1[1]; g[6] = g1[2]; g[7] = g1[3];
  }
  if constexpr (MASK == 3 || MASK == 5) {
    // + the MaxPool2d(2, 2) backward: the pooled grad goes to the window's
    // first max (rr_maxpool2_bwd's routing), added before the ReLU mask
    const int C = a.C;
    const int r = (int)(e / C), c = (int)(e - (long long)r * C);
    const int hw = a.h * a.w;
    const int nn = r / hw, rem = r - nn * hw, y = rem / a.w, x = rem - y * a.w;
    const long long op = ((long long)nn * (a.h >> 1) + (y >> 1)) * (a.w >> 1) + (x >> 1);
    const int k = ((y & 1) << 1) | (x & 1);
    const uint2 id = *reinterpret_cast<const uint2 *>(a.pidx + op * C + c);
    f32x4 p0, p1;
    load8<T>((const T *)a.pdy + op * C + c, p0, p1);
    const float pv[8] = {p0[0], p0[1], p0[2], p0[3], p1[0], p1[1], p1[2], p1[3]};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ij = (int)(((j < 4 ? id.x : id.y) >> (8 * (j & 3))) & 0xff);
      g[j] += ij == k ? pv[j] : 0.f;
    }
  }
  if constexpr (MASK == 4 || MASK == 5) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4 v = f32x4{tA[4 * h], tA[4 * h + 1], tA[4 * h + 2], tA[4 * h + 3]};
      f32x4 q = f32x4{tB[4 * h], tB[4 * h + 1], tB[4 * h + 2], tB[4 * h + 3]};
      const f32x4 sv = f32x4{s8[4 * h], s8[4 * h + 1], s8[4 * h + 2], s8[4 * h + 3]};
      const f32x4 bv = f32x4{b8[4 * h], b8[4 * h + 1], b8[4 * h + 2], b8[4 * h + 3]};
      const f32x4 sq = f32x4{sB[4 * h], sB[4 * h + 1], sB[4 * h + 2], sB[4 * h + 3]};
      const f32x4 bq = f32x4{bB[4 * h], bB[4 * h + 1], bB[4 * h + 2], bB[4 * h + 3]};
      v = v * sv + bv;
      q = q * sq + bq;
      v += q;
#pragma unroll
      for (int k = 0; k < 4; ++k) g[4 * h + k] = fmaxf(v[k], 0.f) > 0.f ? g[4 * h + k] : 0.f;
    }
  } else if constexpr (MASK == 1 || MASK == 3) {
    f32x4 m0, m1;
    load8<T>((const T *)a.aux + e, m0, m1);
    const float m[8] = {m0[0], m0[1], m0[2], m0[3], m1[0], m1[1], m1[2], m1[3]};
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = m[k] > 0.f ? g[k] : 0.f;
  } else if constexpr (MASK == 2) {
    f32x4 t0, t1;
    load8<T>((const T *)a.aux + e, t0, t1);
    const float t[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float u = t[k] * s8[k] + b8[k];
      ag += u > 0.f ? 0.f : g[k] * u;
      g[k] = u > 0.f ? g[k] : al * g[k];
    }
  }
}

// GMO: gm (the masked upstream grad) is also stored, rounded to T, and the
// sums are taken over the stored values -- the apply then reads gm alone
// (rr_bn_bwd_reduce_gm: the identity-shortcut tail, whose gm is the block's
// input grad anyway)
template <typename T, int MASK, int NBN, bool GMO = false>
__global__ __launch_bounds__(256) void bn_bwd_reduce8_kernel(BnBwd a, float *__restrict__ part,
                                                             float *__restrict__ apart,
                                                             long long rows_per_block,
                                                             T *__restrict__ gmo = nullptr) {
  extern __shared__ __attribute__((aligned(16))) float sm[];   // [R][C][3] + [256]
  const int TPR = a.C / 8;
  const int R = 256 / TPR;
  const int tr = threadIdx.x / TPR, tc = threadIdx.x % TPR;
  const int c = tc * 8;
  constexpr bool AFF = MASK == 2 || MASK >= 4, REC = MASK >= 4;
  float m0[8], i0[8], m1[8], i1[8], s8[8], b8[8], sB[8], bB[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    m0[k] = a.mean0[c + k]; i0[k] = a.inv0[c + k];
    m1[k] = NBN == 2 ? a.mean1[c + k] : 0.f; i1[k] = NBN == 2 ? a.inv1[c + k] : 0.f;
    s8[k] = AFF ? a.aff_s[c + k] : 0.f; b8[k] = AFF ? a.aff_b[c + k] : 0.f;
    sB[k] = REC ? a.aff_s[a.C + c + k] : 0.f; bB[k] = REC ? a.aff_b[a.C + c + k] : 0.f;
  }
  const float al = MASK == 2 ? a.alpha[0] : 0.f;
  float s[3][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s[0][k] = 0.f; s[1][k] = 0.f; s[2][k] = 0.f; }
  float asum = 0.f;
  const long long r0 = blockIdx.x * rows_per_block;
  const long long r1 = min(a.P, r0 + rows_per_block);
  // 2 rows per trip: the second row's loads issue before the first row's
  // math (no stores in the loop, so nothing orders them); same add order
#pragma unroll 2
  for (long long r = r0 + tr; r < r1; r += R) {
    const long long e = r * a.C + c;
    float gm[8], t0[8], t1[8];
    f32x4 u0, u1;
    load8<T>((const T *)a.t0 + e, u0, u1);
    t0[0] = u0[0]; t0[1] = u0[1]; t0[2] = u0[2]; t0[3] = u0[3];
    t0[4] = u1[0]; t0[5] = u1[1]; t0[6] = u1[2]; t0[7] = u1[3];
    if constexpr (NBN == 2) {
      load8<T>((const T *)a.t1 + e, u0, u1);
      t1[0] = u0[0]; t1[1] = u0[1]; t1[2] = u0[2]; t1[3] = u0[3];
      t1[4] = u1[0]; t1[5] = u1[1]; t1[6] = u1[2]; t1[7] = u1[3];
    }
    bwd_gm8<T, MASK>(a, e, s8, b8, al, gm, asum, t0, t1, sB, bB);
    if constexpr (GMO) {
#pragma unroll
      for (int k = 0; k < 8; ++k) gm[k] = Elt<T>::round(gm[k]);
      store8<T>(gmo + e, f32x4{gm[0], gm[1], gm[2], gm[3]}, f32x4{gm[4], gm[5], gm[6], gm[7]});
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s[0][k] += gm[k];
      s[1][k] += gm[k] * ((t0[k] - m0[k]) * i0[k]);
    }
    if constexpr (NBN == 2) {
#pragma unroll
      for (int k = 0; k < 8; ++k) s[2][k] += gm[k] * ((t1[k] - m1[k]) * i1[k]);
    }
  }
  float *red = sm;                       // [R][C][3]
  float *ared = sm + (size_t)R * a.C * 3;
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int j = 0; j < 3; ++j) red[((size_t)tr * a.C + c + k) * 3 + j] = s[j][k];
  ared[threadIdx.x] = asum;
  __syncthreads();
  for (int i = threadIdx.x; i < a.C * 3; i += blockDim.x) {
    float v = 0.f;
    for (int rr = 0; rr < R; ++rr) v += red[(size_t)rr * a.C * 3 + i];
    part[(long long)blockIdx.x * a.C * 3 + i] = v;
  }
  if (apart && threadIdx.x == 0) {
    float v = 0.f;
    for (int i = 0; i < (int)blockDim.x; ++i) v += ared[i];
    apart[blockIdx.x] = v;
  }
}

// GCO: g recomputed from the final 1x1 conv's output grad (a.cody, a.cow:
// 3 output channels), rounded to T as rr_conv_out_bwd would have stored it
template <typename T, int MASK, int NBN, bool GMO, bool GCO = false>
__global__ __launch_bounds__(256) void bn_bwd_apply8_kernel(BnBwd a, const float *__restrict__ coef,
                                                            T *dt0, T *dt1, T *gmo) {
  const int G = a.C / 8;
  const int c = (threadIdx.x % G) * 8;   // fixed: G divides the grid stride
  constexpr bool AFF = MASK == 2 || MASK >= 4, REC = MASK >= 4;
  // dt = c0 (gm - c1 - (t - mu) inv c2) folded to dt = A gm + B t + D: three
  // per-channel constants per BN in registers instead of five (the NBN = 2
  // variants sat at 162-172 VGPRs, 2-3 waves per SIMD)
  // the recomputed-mask affines (MASK 4/5: four per channel) are read from
  // LDS per row instead of held in registers
  float fA[2][8], fB[2][8], fD[2][8], s8[8], b8[8], sB[8], bB[8];
  __shared__ __attribute__((aligned(16))) float rcs[REC ? 4 * 1024 : 4];
  if constexpr (REC) {
    for (int i = threadIdx.x; i < a.C; i += blockDim.x) {
      rcs[i] = a.aff_s[i]; rcs[1024 + i] = a.aff_b[i];
      rcs[2048 + i] = a.aff_s[a.C + i]; rcs[3072 + i] = a.aff_b[a.C + i];
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float c0 = 0.f, c1 = 0.f, c2 = 0.f, mu = 0.f, iv = 0.f;
      if (b < NBN) {
        c0 = coef[(c + k) * 6 + 3 * b]; c1 = coef[(c + k) * 6 + 3 * b + 1];
        c2 = coef[(c + k) * 6 + 3 * b + 2];
        mu = (b == 0 ? a.mean0 : a.mean1)[c + k]; iv = (b == 0 ? a.inv0 : a.inv1)[c + k];
      }
      const float q = c0 * c2 * iv;
      fA[b][k] = c0;
      fB[b][k] = -q;
      fD[b][k] = fmaf(q, mu, -c0 * c1);
    }
    s8[k] = AFF && !REC ? a.aff_s[c + k] : 0.f; b8[k] = AFF && !REC ? a.aff_b[c + k] : 0.f;
    sB[k] = 0.f; bB[k] = 0.f;
  }
  const float al = MASK == 2 ? a.alpha[0] : 0.f;
  float cw[GCO ? 3 : 1][8];
  if constexpr (GCO) {
#pragma unroll
    for (int co = 0; co < 3; ++co)
#pragma unroll
      for (int k = 0; k < 8; ++k) cw[co][k] = a.cow[co * a.C + c + k];
  }
  const long long hw = (long long)a.h * a.w;
  const long long rows = a.P;
  const long long stride = ((long long)gridDim.x * blockDim.x) / G;
  for (long long r = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / G; r < rows; r += stride) {
    const long long e = r * a.C + c;
    float gm[8], ag = 0.f, tv[2][8];
    if constexpr (GCO) {
      const long long nn = r / hw, rr = r - nn * hw;
      float d[3];
#pragma unroll
      for (int co = 0; co < 3; ++co) d[co] = a.cody[(nn * 3 + co) * hw + rr];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float t = 0.f;
#pragma unroll
        for (int co = 0; co < 3; ++co) t += d[co] * cw[co][k];
        gm[k] = Elt<T>::round(t);
      }
    }
#pragma unroll
    for (int b = 0; b < NBN; ++b) {
      f32x4 u0, u1;
      load8<T>((const T *)(b == 0 ? a.t0 : a.t1) + e, u0, u1);
      tv[b][0] = u0[0]; tv[b][1] = u0[1]; tv[b][2] = u0[2]; tv[b][3] = u0[3];
      tv[b][4] = u1[0]; tv[b][5] = u1[1]; tv[b][6] = u1[2]; tv[b][7] = u1[3];
    }
    if constexpr (REC) {
      float l[4][8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 u = *reinterpret_cast<const f32x4 *>(rcs + 1024 * j + c);
        const f32x4 v = *reinterpret_cast<const f32x4 *>(rcs + 1024 * j + c + 4);
        l[j][0] = u[0]; l[j][1] = u[1]; l[j][2] = u[2]; l[j][3] = u[3];
        l[j][4] = v[0]; l[j][5] = v[1]; l[j][6] = v[2]; l[j][7] = v[3];
      }
      bwd_gm8<T, MASK, GCO>(a, e, l[0], l[1], al, gm, ag, tv[0], tv[NBN - 1], l[2], l[3]);
    } else {
      bwd_gm8<T, MASK, GCO>(a, e, s8, b8, al, gm, ag, tv[0], tv[NBN - 1], sB, bB);
    }
    if constexpr (GMO)
      store8<T>(gmo + e, f32x4{gm[0], gm[1], gm[2], gm[3]}, f32x4{gm[4], gm[5], gm[6], gm[7]});
#pragma unroll
    for (int b = 0; b < NBN; ++b) {
      const float *t = tv[b];
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaf(fB[b][k], t[k], fmaf(fA[b][k], gm[k], fD[b][k]));
      store8<T>((b == 0 ? dt0 : dt1) + e, f32x4{o[0], o[1], o[2], o[3]}, f32x4{o[4], o[5], o[6], o[7]});
    }
  }
}

// rows of [P][C] handled by one workgroup: TPR = C/4 threads per row
template <typename T>
__global__ void bn_bwd_reduce_kernel(BnBwd a, float *__restrict__ part, float *__restrict__ apart,
                                     long long rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) float sm[];   // [R][C][3] + [256]
  const int TPR = a.C / 4;
  const int R = blockDim.x / TPR;
  const int tr = threadIdx.x / TPR, tc = threadIdx.x % TPR;
  const int c = tc * 4;
  float s[3][4] = {{0.f}};
  float asum = 0.f;
  const long long r0 = blockIdx.x * rows_per_block;
  const long long r1 = min(a.P, r0 + rows_per_block);
  if (tr < R) {
    for (long long r = r0 + tr; r < r1; r += R) {
      const long long e = r * a.C + c;
      f32x4 ag;
      const f32x4 gm = bwd_gm<T>(a, e, c, ag);
      const f32x4 t0 = load4<T>((const T *)a.t0 + e);
      const f32x4 m0 = *reinterpret_cast<const f32x4 *>(a.mean0 + c);
      const f32x4 i0 = *reinterpret_cast<const f32x4 *>(a.inv0 + c);
      f32x4 t1 = {0.f, 0.f, 0.f, 0.f}, m1 = t1, i1 = t1;
      if (a.nbn == 2) {
        t1 = load4<T>((const T *)a.t1 + e);
        m1 = *reinterpret_cast<const f32x4 *>(a.mean1 + c);
        i1 = *reinterpret_cast<const f32x4 *>(a.inv1 + c);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s[0][k] += gm[k];
        s[1][k] += gm[k] * ((t0[k] - m0[k]) * i0[k]);
        s[2][k] += gm[k] * ((t1[k] - m1[k]) * i1[k]);
        asum += ag[k];
      }
    }
  }
  float *red = sm;                       // [R][C][3]
  float *ared = sm + (size_t)R * a.C * 3;
  if (tr < R) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 3; ++j) red[((size_t)tr * a.C + c + k) * 3 + j] = s[j][k];
  }
  ared[threadIdx.x] = asum;
  __syncthreads();
  for (int i = threadIdx.x; i < a.C * 3; i += blockDim.x) {
    float v = 0.f;
    for (int rr = 0; rr < R; ++rr) v += red[(size_t)rr * a.C * 3 + i];
    part[(long long)blockIdx.x * a.C * 3 + i] = v;
  }
  if (apart && threadIdx.x == 0) {
    float v = 0.f;
    for (int i = 0; i < (int)blockDim.x; ++i) v += ared[i];
    apart[blockIdx.x] = v;
  }
}

// coef[C][2][3] = {gamma*invstd, mean(gm), mean(gm*xhat)} per BN
// one workgroup per channel: 256 row lanes sum the partial rows in a fixed
// order, then a fixed LDS tree (the old 16-channel blocks left most of the
// chip idle on <= 1024 rows: 18.6 us at C = 64)
template <typename PT>
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(
    int C, int blocks, double count, int nbn, const PT *__restrict__ part, int ablocks,
    const float *apart, const float *g0, const float *inv0, const float *g1, const float *inv1,
    float *dg0, float *db0, float *dg1, float *db1, float *dalpha, float *coef, float *dbias0,
    float *dbias1) {
  __shared__ double red[3][256];
  const int c = blockIdx.x, t = threadIdx.x;
  double s[3] = {0, 0, 0};
  rr_fixed_sum<3>(part + ((long long)t * C + c) * 3, 256LL * C * 3, rr_trips(t, blocks, 256), s);
  double s0 = s[0], s1 = s[1], s2 = s[2];
  red[0][t] = s0; red[1][t] = s1; red[2][t] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      red[0][t] += red[0][t + o];
      red[1][t] += red[1][t + o];
      red[2][t] += red[2][t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    s0 = red[0][0]; s1 = red[1][0]; s2 = red[2][0];
    if (db0) db0[c] = (float)s0;
    if (dg0) dg0[c] = (float)s1;
    // eval mode: count = +inf, so the batch-statistic terms are exactly 0
    coef[c * 6 + 0] = (g0 ? g0[c] : 1.f) * inv0[c];
    coef[c * 6 + 1] = (float)(s0 / count);
    coef[c * 6 + 2] = (float)(s1 / count);
    if (dbias0) dbias0[c] = coef[c * 6 + 0] * (float)s0;
    if (nbn == 2) {
      if (db1) db1[c] = (float)s0;
      if (dg1) dg1[c] = (float)s2;
      coef[c * 6 + 3] = (g1 ? g1[c] : 1.f) * inv1[c];
      coef[c * 6 + 4] = (float)(s0 / count);
      coef[c * 6 + 5] = (float)(s2 / count);
      if (dbias1) dbias1[c] = coef[c * 6 + 3] * (float)s0;
    }
  }
  if (blockIdx.x == 0 && apart && dalpha) {
    __syncthreads();
    double v[1] = {0};
    rr_fixed_sum<1>(apart + t, 256, rr_trips(t, ablocks, 256), v);
    red[0][t] = v[0];
    __syncthreads();
    if (t == 0) {
      double tt = 0;
      for (int i = 0; i < 256; ++i) tt += red[0][i];
      dalpha[0] = (float)tt;
    }
  }
}

template <typename T>
__global__ void bn_bwd_apply_kernel(BnBwd a, const float *__restrict__ coef, T *dt0, T *dt1,
                                    T *gmo) {
  const long long n4 = a.P * a.C / 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    const long long e = i * 4;
    const int c = (int)(e % a.C);
    f32x4 ag;
    const f32x4 gm = bwd_gm<T>(a, e, c, ag);
    if (gmo) store4<T>(gmo + e, gm);
    {
      const f32x4 t = load4<T>((const T *)a.t0 + e);
      f32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float *cf = coef + (c + k) * 6;
        const float xh = (t[k] - a.mean0[c + k]) * a.inv0[c + k];
        o[k] = cf[0] * (gm[k] - cf[1] - xh * cf[2]);
      }
      store4<T>(dt0 + e, o);
    }
    if (a.nbn == 2) {
      const f32x4 t = load4<T>((const T *)a.t1 + e);
      f32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float *cf = coef + (c + k) * 6 + 3;
        const float xh = (t[k] - a.mean1[c + k]) * a.inv1[c + k];
        o[k] = cf[0] * (gm[k] - cf[1] - xh * cf[2]);
      }
      store4<T>(dt1 + e, o);
    }
  }
}

// ---------------------------------------------------------------------------
// column sums (bias grads): partial [blocks][C] then finalize (fixed order)
template <typename T>
__global__ void colsum_kernel(long long P, int C, const T *__restrict__ x, float *__restrict__ part,
                              long long rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int TPR = C / 4;
  const int R = blockDim.x / TPR;
  const int tr = threadIdx.x / TPR, tc = threadIdx.x % TPR;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  const long long r0 = blockIdx.x * rows_per_block;
  const long long r1 = min(P, r0 + rows_per_block);
  if (tr < R) {
#pragma unroll 4
    for (long long r = r0 + tr; r < r1; r += R) {
      const f32x4 v = load4<T>(x + r * C + tc * 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) s[k] += v[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) sm[(size_t)tr * C + tc * 4 + k] = s[k];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    float v = 0.f;
    for (int rr = 0; rr < R; ++rr) v += sm[(size_t)rr * C + i];
    part[(long long)blockIdx.x * C + i] = v;
  }
}

__global__ void colsum_finalize(int C, int blocks, const float *__restrict__ part, float *out,
                                int accumulate) {
  __shared__ double red[16][17];
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double sv[1] = {0};
  if (c < C) rr_fixed_sum<1>(part + (long long)sl * C + c, 16LL * C, rr_trips(sl, blocks, 16), sv);
  double s = sv[0];
  red[sl][cl] = s;
  __syncthreads();
  if (sl == 0 && c < C) {
    for (int k = 1; k < 16; ++k) s += red[k][cl];
    out[c] = accumulate ? out[c] + (float)s : (float)s;
  }
}

// per-block (sum, sum of squares) of a [P][C] tensor: the batch statistics of
// a standalone BatchNorm2d (leaf-module path, nn.py) when no conv epilogue
// produced them.  partial [blocks][C][2], the layout rr_bn_finalize reads.
template <typename T>
__global__ void colstats_kernel(long long P, int C, const T *__restrict__ x, float *__restrict__ part,
                                long long rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) float sm[];   // [R][C][2]
  const int TPR = C / 4;
  const int R = blockDim.x / TPR;
  const int tr = threadIdx.x / TPR, tc = threadIdx.x % TPR;
  float s[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
  const long long r0 = blockIdx.x * rows_per_block;
  const long long r1 = min(P, r0 + rows_per_block);
  if (tr < R) {
#pragma unroll 4
    for (long long r = r0 + tr; r < r1; r += R) {
      const f32x4 v = load4<T>(x + r * C + tc * 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) { s[k] += v[k]; q[k] = fmaf(v[k], v[k], q[k]); }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sm[((size_t)tr * C + tc * 4 + k) * 2] = s[k];
      sm[((size_t)tr * C + tc * 4 + k) * 2 + 1] = q[k];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < R; ++rr) { a += sm[((size_t)rr * C + i) * 2]; b += sm[((size_t)rr * C + i) * 2 + 1]; }
    part[((long long)blockIdx.x * C + i) * 2] = a;
    part[((long long)blockIdx.x * C + i) * 2 + 1] = b;
  }
}

int reduce_blocks(long long P) {
  long long b = (P + 63) / 64;
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

// the direct path (<= RR_BN_DIRECT_ROWS partial rows) reads the partials in
// place and needs no workspace
#define RR_BN_DIRECT_ROWS 8192
extern "C" size_t rr_bn_finalize_workspace(int C, int blocks) {
  return blocks <= RR_BN_DIRECT_ROWS ? 0 : rr_colreduce_bytes(blocks, C * 2);
}

extern "C" int rr_bn_finalize(int C, int blocks, long long count, const float *part,
                              const float *bias, const float *gamma, const float *beta,
                              float *running_mean, float *running_var, float momentum,
                              float eps, float *scale, float *shift, float *save_mean,
                              float *save_invstd, int64_t *num_batches_tracked, void *ws,
                              size_t ws_bytes, rr_stream stream) {
  if (C <= 0 || blocks <= 0 || count <= 0 || !part || !scale || !shift) return RR_EINVAL;
  const bool cum = momentum < 0.f;
  if (cum && !num_batches_tracked) return RR_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (blocks <= RR_BN_DIRECT_ROWS) {
    hipLaunchKernelGGL(bn_finalize_direct_kernel, dim3(C), dim3(256), 0, st, C, blocks, (double)count,
                       part, bias, gamma, beta, running_mean, running_var, momentum, eps, scale, shift,
                       save_mean, save_invstd, num_batches_tracked);
    RR_CHECK_LAUNCH();
  } else {
    if (!ws || ws_bytes < rr_colreduce_bytes(blocks, C * 2)) return RR_EWORKSPACE;
    const int chunks = rr_colreduce(part, blocks, C * 2, (double *)ws, st);
    if (chunks < 0) return RR_ELAUNCH;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, st,
                       C, chunks, (double)count, (const double *)ws, bias, gamma, beta, running_mean,
                       running_var, momentum, eps, scale, shift, save_mean, save_invstd,
                       num_batches_tracked);
    RR_CHECK_LAUNCH();
  }
  if (cum) {
    hipLaunchKernelGGL(bn_nbt_inc_kernel, dim3(1), dim3(1), 0, st, num_batches_tracked);
    RR_CHECK_LAUNCH();
  }
  return RR_OK;
}

// two BatchNorms in one launch (direct path only: both with <= 8192 partial
// rows; else RR_EUNSUPPORTED and the caller finalizes them separately)
extern "C" int rr_bn_finalize_pair(const rr_bn_finalize_desc *a, const rr_bn_finalize_desc *b,
                                   rr_stream stream) {
  if (!a || !b) return RR_EINVAL;
  for (const rr_bn_finalize_desc *d : {a, b})
    if (d->C <= 0 || d->blocks <= 0 || d->count <= 0 || !d->part || !d->scale || !d->shift)
      return RR_EINVAL;
  if (a->blocks > RR_BN_DIRECT_ROWS || b->blocks > RR_BN_DIRECT_ROWS) return RR_EUNSUPPORTED;
  if (a->momentum < 0.f || b->momentum < 0.f) return RR_EUNSUPPORTED;   // cumulative: rr_bn_finalize
  auto fin = [](const rr_bn_finalize_desc *d) {
    return BnFin{d->C, d->blocks, (double)d->count, d->part, d->bias, d->gamma, d->beta,
                 d->running_mean, d->running_var, d->momentum, d->eps, d->scale, d->shift,
                 d->save_mean, d->save_invstd, d->num_batches_tracked};
  };
  hipLaunchKernelGGL(bn_finalize_direct2_kernel, dim3(a->C + b->C), dim3(256), 0, (hipStream_t)stream,
                     fin(a), fin(b));
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" int rr_bn_eval_affine(int C, const float *gamma, const float *beta,
                                 const float *running_mean, const float *running_var, float eps,
                                 float *scale, float *shift, rr_stream stream) {
  if (C <= 0 || !running_mean || !running_var || !scale || !shift) return RR_EINVAL;
  hipLaunchKernelGGL(bn_eval_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     C, gamma, beta, running_mean, running_var, eps, scale, shift);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

// eval-mode BatchNorm folded into the conv before it (17:84-85 inference):
// BN(W x + b) = (s W) x + (s b + t) with s, t = rr_bn_eval_affine's scale /
// shift; w [co][kel] fp32 (torch layout, kel = c_in * k * k)
__global__ void fold_conv_bn_kernel(int co, int kel, const float *__restrict__ w,
                                    const float *__restrict__ b, const float *__restrict__ scale,
                                    const float *__restrict__ shift, float *__restrict__ w_out,
                                    float *__restrict__ b_out) {
  const long long total = (long long)co * kel;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i / kel);
    w_out[i] = w[i] * scale[c];
    if (i - (long long)c * kel == 0) b_out[c] = (b ? b[c] : 0.f) * scale[c] + shift[c];
  }
}

extern "C" int rr_fold_conv_bn(int co, int kel, const float *w, const float *b, const float *scale,
                               const float *shift, float *w_out, float *b_out, rr_stream stream) {
  if (co <= 0 || kel <= 0 || !w || !scale || !shift || !w_out || !b_out) return RR_EINVAL;
  const long long total = (long long)co * kel;
  hipLaunchKernelGGL(fold_conv_bn_kernel, dim3(rr_grid_cap((total + 255) / 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, co, kel, w, b, scale, shift, w_out, b_out);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" int rr_affine_act(int dtype, long long P, int C, const void *x, const float *scale,
                             const float *shift, const float *alpha, const void *res,
                             const float *res_scale, const float *res_shift, int relu, void *y,
                             rr_stream stream) {
  if (P <= 0 || C <= 0 || C % 4 || !x || !scale || !shift || !y) return RR_EINVAL;
  if ((res_scale == nullptr) != (res_shift == nullptr)) return RR_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (C % 8 == 0 && 256 % (C / 8) == 0) {
    const int grid8 = rr_grid_cap((P * C / 8 + 255) / 256, RR_EW_GRID);
    if (dtype == RR_BF16)
      hipLaunchKernelGGL(affine_act8_kernel<bf16_t>, dim3(grid8), dim3(256), 0, st, P, C,
                         (const bf16_t *)x, scale, shift, alpha, (const bf16_t *)res, res_scale,
                         res_shift, relu, (bf16_t *)y);
    else
      hipLaunchKernelGGL(affine_act8_kernel<float>, dim3(grid8), dim3(256), 0, st, P, C,
                         (const float *)x, scale, shift, alpha, (const float *)res, res_scale,
                         res_shift, relu, (float *)y);
    RR_CHECK_LAUNCH();
    return RR_OK;
  }
  const int grid = rr_grid_cap((P * C / 4 + 255) / 256, 4096);
  if (dtype == RR_BF16)
    hipLaunchKernelGGL(affine_act_kernel<bf16_t>, dim3(grid), dim3(256), 0, st, P, C,
                       (const bf16_t *)x, scale, shift, alpha, (const bf16_t *)res, res_scale,
                       res_shift, relu, (bf16_t *)y);
  else
    hipLaunchKernelGGL(affine_act_kernel<float>, dim3(grid), dim3(256), 0, st, P, C,
                       (const float *)x, scale, shift, alpha, (const float *)res, res_scale,
                       res_shift, relu, (float *)y);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" int rr_affine_act_pool(int dtype, int n, int h, int w, int C, const void *x,
                                  const float *scale, const float *shift, const void *res,
                                  const float *res_scale, const float *res_shift, int relu, void *y,
                                  void *y_pool, uint8_t *idx, rr_stream stream) {
  if (n <= 0 || h <= 0 || w <= 0 || h % 2 || w % 2 || C <= 0 || C % 8 || !x || !scale || !shift ||
      !y || !y_pool || !idx)
    return RR_EINVAL;
  if ((res_scale == nullptr) != (res_shift == nullptr) || (res_scale && !res)) return RR_EINVAL;
  const long long total = (long long)n * (h / 2) * (w / 2) * (C / 8);
  const int grid = rr_grid_cap((total + 255) / 256, 8192);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RR_BF16)
    hipLaunchKernelGGL(affine_act_pool_kernel<bf16_t>, dim3(grid), dim3(256), 0, st, n, h, w, C,
                       (const bf16_t *)x, scale, shift, (const bf16_t *)res, res_scale, res_shift, relu,
                       (bf16_t *)y, (bf16_t *)y_pool, idx);
  else
    hipLaunchKernelGGL(affine_act_pool_kernel<float>, dim3(grid), dim3(256), 0, st, n, h, w, C,
                       (const float *)x, scale, shift, (const float *)res, res_scale, res_shift, relu,
                       (float *)y, (float *)y_pool, idx);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" int rr_bn_bwd_blocks(const rr_bnbwd_desc *d) {
  if (!d) return RR_EINVAL;
  return reduce_blocks(d->P);
}

// the sample count of the batch-statistic terms; eval mode: +inf (the terms vanish)
static double bnbwd_count(const rr_bnbwd_desc *d) {
  return d->eval ? __builtin_huge_val() : (double)d->P;
}

static int bnbwd_check(const rr_bnbwd_desc *d) {
  if (!d || d->P <= 0 || d->C <= 0 || d->C % 4 || d->C / 4 > 256) return RR_EINVAL;
  if (d->nbn != 1 && d->nbn != 2) return RR_EINVAL;
  if (d->mask_kind < 0 || d->mask_kind > 5) return RR_EINVAL;
  if (d->mask_kind >= 4 && (d->nbn != 2 || d->C % 8 || 256 % (d->C / 8)))
    return RR_EUNSUPPORTED;                 // recomputed mask: BN shortcut, 8-channel kernels
  if (d->mask_kind == 3 || d->mask_kind == 5) {
    if (!d->pool_dy || !d->pool_idx || d->h <= 0 || d->w <= 0 || d->h % 2 || d->w % 2 ||
        d->P % ((long long)d->h * d->w) || d->C % 8 || 256 % (d->C / 8) || d->P > 0x7fffffffLL)
      return RR_EUNSUPPORTED;               // 8-channel kernels only
  }
  return RR_OK;
}

static BnBwd make_bnbwd(const rr_bnbwd_desc *d, const void *g, const void *aux,
                        const float *aff_s, const float *aff_b, const float *alpha,
                        const void *t0, const float *mean0, const float *inv0, const void *t1,
                        const float *mean1, const float *inv1) {
  BnBwd a;
  a.P = d->P; a.C = d->C; a.mask_kind = d->mask_kind; a.nbn = d->nbn;
  a.h = d->h; a.w = d->w; a.pdy = d->pool_dy; a.pidx = d->pool_idx;
  a.g = g; a.aux = aux; a.aff_s = aff_s; a.aff_b = aff_b; a.alpha = alpha;
  a.t0 = t0; a.t1 = t1; a.mean0 = mean0; a.inv0 = inv0; a.mean1 = mean1; a.inv1 = inv1;
  a.cody = nullptr; a.cow = nullptr;
  return a;
}

extern "C" int rr_bn_bwd_reduce(const rr_bnbwd_desc *d, const void *g, const void *aux,
                                const float *aff_s, const float *aff_b, const float *alpha,
                                const void *t0, const float *mean0, const float *invstd0,
                                const void *t1, const float *mean1, const float *invstd1,
                                float *partial, rr_stream stream) {
  int rc = bnbwd_check(d);
  if (rc) return rc;
  if (!g || !t0 || !mean0 || !invstd0 || !partial) return RR_EINVAL;
  if (d->mask_kind && d->mask_kind < 4 && !aux) return RR_EINVAL;
  if (d->mask_kind == 2 && (!aff_s || !aff_b || !alpha)) return RR_EINVAL;
  if (d->mask_kind >= 4 && (!aff_s || !aff_b)) return RR_EINVAL;
  if (d->nbn == 2 && (!t1 || !mean1 || !invstd1)) return RR_EINVAL;
  const BnBwd a = make_bnbwd(d, g, aux, aff_s, aff_b, alpha, t0, mean0, invstd0, t1, mean1, invstd1);
  const int blocks = reduce_blocks(d->P);
  const long long rpb = (d->P + blocks - 1) / blocks;
  const int TPR = d->C / 4;
  const int R = 256 / TPR;
  const size_t shm = ((size_t)R * d->C * 3 + 256) * sizeof(float);
  float *apart = partial + (size_t)blocks * d->C * 3;
  hipStream_t st = (hipStream_t)stream;
  if (d->C % 8 == 0 && 256 % (d->C / 8) == 0) {
    const size_t shm8 = ((size_t)(256 / (d->C / 8)) * d->C * 3 + 256) * sizeof(float);
    float *ap = d->mask_kind == 2 ? apart : nullptr;
#define RR_RED8(TT, M, N) hipLaunchKernelGGL((bn_bwd_reduce8_kernel<TT, M, N>), dim3(blocks), dim3(256), shm8, st, a, partial, ap, rpb)
#define RR_RED8_T(TT)                                             \
    switch (d->mask_kind * 2 + (d->nbn - 1)) {                    \
      case 0: RR_RED8(TT, 0, 1); break; case 1: RR_RED8(TT, 0, 2); break; \
      case 2: RR_RED8(TT, 1, 1); break; case 3: RR_RED8(TT, 1, 2); break; \
      case 4: RR_RED8(TT, 2, 1); break; case 5: RR_RED8(TT, 2, 2); break; \
      case 6: RR_RED8(TT, 3, 1); break; case 7: RR_RED8(TT, 3, 2); break; \
      case 9: RR_RED8(TT, 4, 2); break; default: RR_RED8(TT, 5, 2); break; \
    }
    if (d->dtype == RR_BF16) { RR_RED8_T(bf16_t) } else { RR_RED8_T(float) }
#undef RR_RED8_T
#undef RR_RED8
    RR_CHECK_LAUNCH();
    return RR_OK;
  }
  if (d->dtype == RR_BF16)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<bf16_t>, dim3(blocks), dim3(256), shm, st, a, partial,
                       d->mask_kind == 2 ? apart : nullptr, rpb);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<float>, dim3(blocks), dim3(256), shm, st, a, partial,
                       d->mask_kind == 2 ? apart : nullptr, rpb);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" int rr_bn_bwd_reduce_gm(const rr_bnbwd_desc *d, const void *g, const void *aux,
                                   const void *t0, const float *mean0, const float *invstd0,
                                   float *partial, void *gm_out, rr_stream stream) {
  int rc = bnbwd_check(d);
  if (rc) return rc;
  if (!g || !aux || !t0 || !mean0 || !invstd0 || !partial || !gm_out) return RR_EINVAL;
  if (d->nbn != 1 || (d->mask_kind != 1 && d->mask_kind != 3) || d->C % 8 || 256 % (d->C / 8))
    return RR_EUNSUPPORTED;
  const BnBwd a = make_bnbwd(d, g, aux, nullptr, nullptr, nullptr, t0, mean0, invstd0, nullptr,
                             nullptr, nullptr);
  const int blocks = reduce_blocks(d->P);
  const long long rpb = (d->P + blocks - 1) / blocks;
  const size_t shm8 = ((size_t)(256 / (d->C / 8)) * d->C * 3 + 256) * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
#define RR_REDGM(TT, M) hipLaunchKernelGGL((bn_bwd_reduce8_kernel<TT, M, 1, true>), dim3(blocks), dim3(256), shm8, st, a, partial, nullptr, rpb, (TT *)gm_out)
  if (d->dtype == RR_BF16) {
    if (d->mask_kind == 1) RR_REDGM(bf16_t, 1); else RR_REDGM(bf16_t, 3);
  } else {
    if (d->mask_kind == 1) RR_REDGM(float, 1); else RR_REDGM(float, 3);
  }
#undef RR_REDGM
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" int rr_bn_bwd_finalize(const rr_bnbwd_desc *d, const float *partial,
                                  const float *gamma0, const float *invstd0, const float *gamma1,
                                  const float *invstd1, float *dgamma0, float *dbeta0,
                                  float *dgamma1, float *dbeta1, float *dalpha, float *coef,
                                  rr_stream stream) {
  int rc = bnbwd_check(d);
  if (rc) return rc;
  if (!partial || !invstd0 || !coef || (d->nbn == 2 && !invstd1)) return RR_EINVAL;
  const int blocks = reduce_blocks(d->P);
  const float *apart = d->mask_kind == 2 ? partial + (size_t)blocks * d->C * 3 : nullptr;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<float>, dim3(d->C), dim3(256), 0,
                     (hipStream_t)stream, d->C, blocks, bnbwd_count(d), d->nbn, partial, blocks, apart,
                     gamma0, invstd0, gamma1, invstd1, dgamma0, dbeta0, dgamma1, dbeta1, dalpha,
                     coef, d->eval ? d->dbias0 : nullptr, d->eval ? d->dbias1 : nullptr);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" int rr_bn_bwd_apply(const rr_bnbwd_desc *d, const void *g, const void *aux,
                               const float *aff_s, const float *aff_b, const float *alpha,
                               const void *t0, const float *mean0, const float *invstd0,
                               const void *t1, const float *mean1, const float *invstd1,
                               const float *coef, void *dt0, void *dt1, void *gm_out,
                               rr_stream stream) {
  int rc = bnbwd_check(d);
  if (rc) return rc;
  if (!g || !t0 || !coef || !dt0 || (d->nbn == 2 && (!t1 || !dt1))) return RR_EINVAL;
  if (d->mask_kind >= 4 && (!aff_s || !aff_b || gm_out)) return RR_EINVAL;
  const BnBwd a = make_bnbwd(d, g, aux, aff_s, aff_b, alpha, t0, mean0, invstd0, t1, mean1, invstd1);
  hipStream_t st = (hipStream_t)stream;
  if (d->C % 8 == 0 && 256 % (d->C / 8) == 0) {
    const int grid8 = rr_grid_cap((d->P * d->C / 8 + 255) / 256, RR_EW_GRID);
#define RR_APP8(TT, M, N, GM) hipLaunchKernelGGL((bn_bwd_apply8_kernel<TT, M, N, GM>), dim3(grid8), dim3(256), 0, st, a, coef, (TT *)dt0, (TT *)dt1, (TT *)gm_out)
#define RR_APP8_M(TT, M)                                                        \
    if (d->nbn == 1) { if (gm_out) RR_APP8(TT, M, 1, true); else RR_APP8(TT, M, 1, false); } \
    else { if (gm_out) RR_APP8(TT, M, 2, true); else RR_APP8(TT, M, 2, false); }
#define RR_APP8_T(TT)                                                           \
    if (d->mask_kind == 0) { RR_APP8_M(TT, 0) } else if (d->mask_kind == 1) { RR_APP8_M(TT, 1) } \
    else if (d->mask_kind == 2) { RR_APP8_M(TT, 2) } else if (d->mask_kind == 3) { RR_APP8_M(TT, 3) } \
    else if (d->mask_kind == 4) { RR_APP8(TT, 4, 2, false); } else { RR_APP8(TT, 5, 2, false); }
    if (d->dtype == RR_BF16) { RR_APP8_T(bf16_t) } else { RR_APP8_T(float) }
#undef RR_APP8_T
#undef RR_APP8_M
#undef RR_APP8
    RR_CHECK_LAUNCH();
    return RR_OK;
  }
  const int grid = rr_grid_cap((d->P * d->C / 4 + 255) / 256, 4096);
  if (d->dtype == RR_BF16)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<bf16_t>, dim3(grid), dim3(256), 0, st, a, coef,
                       (bf16_t *)dt0, (bf16_t *)dt1, (bf16_t *)gm_out);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, dim3(grid), dim3(256), 0, st, a, coef,
                       (float *)dt0, (float *)dt1, (float *)gm_out);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

// the residual-tail BN backward apply of a block whose output feeds the final
// 1x1 conv (ResUNet dec1, 14:149): g recomputed from that conv's output grad
// (rr_conv_out_bwd_bnred reduced it without storing it); recomputed ReLU mask
// (mask kind 4)
extern "C" int rr_bn_bwd_apply_convout(const rr_bnbwd_desc *d, int h, int w, const float *dy,
                                       const float *wt, int cout, const float *aff_s,
                                       const float *aff_b, const void *t0, const float *mean0,
                                       const float *invstd0, const void *t1, const float *mean1,
                                       const float *invstd1, const float *coef, void *dt0, void *dt1,
                                       rr_stream stream) {
  int rc = bnbwd_check(d);
  if (rc) return rc;
  if (!dy || !wt || !aff_s || !aff_b || !t0 || !t1 || !coef || !dt0 || !dt1 || h <= 0 || w <= 0)
    return RR_EINVAL;
  if (d->mask_kind != 4 || d->nbn != 2 || d->P % ((long long)h * w)) return RR_EINVAL;
  if (cout != 3) return RR_EUNSUPPORTED;
  BnBwd a = make_bnbwd(d, nullptr, nullptr, aff_s, aff_b, nullptr, t0, mean0, invstd0, t1, mean1, invstd1);
  a.h = h; a.w = w; a.cody = dy; a.cow = wt;
  const int grid8 = rr_grid_cap((d->P * d->C / 8 + 255) / 256, RR_EW_GRID);
  hipStream_t st = (hipStream_t)stream;
  if (d->dtype == RR_BF16)
    hipLaunchKernelGGL((bn_bwd_apply8_kernel<bf16_t, 4, 2, false, true>), dim3(grid8), dim3(256), 0, st, a, coef,
                       (bf16_t *)dt0, (bf16_t *)dt1, (bf16_t *)nullptr);
  else
    hipLaunchKernelGGL((bn_bwd_apply8_kernel<float, 4, 2, false, true>), dim3(grid8), dim3(256), 0, st, a, coef,
                       (float *)dt0, (float *)dt1, (float *)nullptr);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" size_t rr_channel_sum_workspace(long long P, int C) {
  return (size_t)reduce_blocks(P) * C * sizeof(float);
}

extern "C" int rr_channel_sum(int dtype, long long P, int C, const void *x, float *out,
                              int accumulate, void *ws, size_t ws_bytes, rr_stream stream) {
  if (P <= 0 || C <= 0 || C % 4 || C / 4 > 256 || !x || !out) return RR_EINVAL;
  const int blocks = reduce_blocks(P);
  if (!ws || ws_bytes < (size_t)blocks * C * sizeof(float)) return RR_EWORKSPACE;
  const long long rpb = (P + blocks - 1) / blocks;
  const int R = 256 / (C / 4);
  const size_t shm = (size_t)R * C * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RR_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, dim3(blocks), dim3(256), shm, st, P, C,
                       (const bf16_t *)x, (float *)ws, rpb);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, dim3(blocks), dim3(256), shm, st, P, C,
                       (const float *)x, (float *)ws, rpb);
  RR_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_finalize, dim3((C + 15) / 16), dim3(256), 0, st, C, blocks,
                     (const float *)ws, out, accumulate);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" int rr_bn_stats_blocks(long long P) { return reduce_blocks(P); }

extern "C" int rr_bn_stats(int dtype, long long P, int C, const void *x, float *partial,
                           rr_stream stream) {
  if (P <= 0 || C <= 0 || C % 4 || C / 4 > 256 || !x || !partial) return RR_EINVAL;
  const int blocks = reduce_blocks(P);
  const long long rpb = (P + blocks - 1) / blocks;
  const int R = 256 / (C / 4);
  const size_t shm = (size_t)R * C * 2 * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RR_BF16)
    hipLaunchKernelGGL(colstats_kernel<bf16_t>, dim3(blocks), dim3(256), shm, st, P, C,
                       (const bf16_t *)x, partial, rpb);
  else
    hipLaunchKernelGGL(colstats_kernel<float>, dim3(blocks), dim3(256), shm, st, P, C,
                       (const float *)x, partial, rpb);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

// at most this many partial rows: the single-launch finalize (measured 5-7 us
// against 4.8 + 5-7 us for the column reduce + finalize pair at 256-1024 rows)
#define RR_BNBWD_DIRECT_ROWS 1024
extern "C" size_t rr_bn_bwd_finalize_rows_workspace(int C, int rows) {
  return rr_colreduce_bytes(rows, C * 3);
}

extern "C" int rr_bn_bwd_finalize_rows(const rr_bnbwd_desc *d, int rows, const float *partial,
                                       int arows, const float *apartial, const float *gamma0,
                                       const float *invstd0, float *dgamma0, float *dbeta0,
                                       float *dalpha, float *coef, void *ws, size_t ws_bytes,
                                       rr_stream stream) {
  int rc = bnbwd_check(d);
  if (rc) return rc;
  if (d->nbn != 1 || rows <= 0 || !partial || !invstd0 || !coef) return RR_EINVAL;
  if ((arows > 0) != (apartial != nullptr)) return RR_EINVAL;
  if (!ws || ws_bytes < rr_colreduce_bytes(rows, d->C * 3)) return RR_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  if (rows <= RR_BNBWD_DIRECT_ROWS) {
    // few rows (the 8x8 / 16x16 maps): the finalize reads the raw rows
    // itself -- one launch instead of the column reduce + finalize pair
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<float>, dim3(d->C), dim3(256), 0, st,
                       d->C, rows, bnbwd_count(d), 1, partial, arows, apartial, gamma0,
                       invstd0, nullptr, nullptr, dgamma0, dbeta0, nullptr, nullptr, dalpha, coef,
                       d->eval ? d->dbias0 : nullptr, nullptr);
    RR_CHECK_LAUNCH();
    return RR_OK;
  }
  const int chunks = rr_colreduce(partial, rows, d->C * 3, (double *)ws, st);
  if (chunks < 0) return RR_ELAUNCH;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<double>, dim3(d->C), dim3(256), 0, st,
                     d->C, chunks, bnbwd_count(d), 1, (const double *)ws, arows, apartial, gamma0,
                     invstd0, nullptr, nullptr, dgamma0, dbeta0, nullptr, nullptr, dalpha, coef,
                     d->eval ? d->dbias0 : nullptr, nullptr);
  RR_CHECK_LAUNCH();
  return RR_OK;
}
