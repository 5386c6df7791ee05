// igemm_epi.h -- the implicit-GEMM argument block and the staged conv
// epilogue shared by the tiled kernels of igemm.hip and the tap-reuse conv
// (conv3r.hip).  Internal; not part of the C ABI.
#pragma once
#include "common.h"

struct IgemmArgs {
  const char *x1, *x2, *wt;
  const float *bias;
  char *y1, *y2;
  const char *mask;
  float *stats;
  int n, h, w;        // GEMM row grid
  int c1, c2, cin;    // K-side channels
  int cout;           // GEMM columns
  int split;          // column split (0: none)
  int act, accumulate, has_mask;
  int taps, K;
  int P;              // n*h*w
  int ncblk;
  int cout_t;         // convT_up: channels per tap
  int out_nchw;       // y1 = fp32 NCHW
  // BN-backward fusion (rr_igemm_bnbwd): the accumulator is dL/d(PReLU out)
  // of a BN -> PReLU pair; the epilogue writes gm = dL/d(BN out) and the
  // per-channel partials of sum(gm), sum(gm * xhat) and the PReLU alpha grad
  const char *bt;                              // pre-BN activation t [P][cout]
  const float *bmean, *binv, *baff_s, *baff_b, *balpha;
  float *bpart, *bapart;                       // [npblk][cout][3], [npblk][cout/64]
  int xcd;            // XCD-aware tile order (RR_XCD_MAP=0 disables)
  // rr_igemm_ex (conv3r register epilogue): PReLU alpha (act & 3 ==
  // RR_ACT_PRELU), residual added before the activation (act & RR_ACT_RES)
  const float *alpha;
  const char *res;
  char *ypool;        // act & RR_ACT_POOL: [n][h/2][w/2][c_out] 2x2 max-pool of the output
  uint8_t *pidx;      // (rr_igemm_pool) its first-max window index, or null
  int ntile;          // conv3r: tiles of the launch (a persistent grid walks them)
};

namespace {


// BN-backward fused epilogue (see IgemmArgs::bpart).  Thread -> fixed
// 8-channel chunk cc; per-thread sums reduced over the lanes sharing cc
// (xor shuffles), then over the waves in LDS (fixed order).
template <typename T, int BC, int BP, int NT>
__device__ __forceinline__ void store_staged_bnbwd(const IgemmArgs &a, float *stg, int c0, int p0,
                                                   int pblk, int tid, int nvalid) {
  constexpr int SROW = BC + 4;
  constexpr int CPR = BC / 8;
  constexpr int NCH = BP * CPR / NT;
  constexpr int NW = NT / 64;
  const int cc = (tid % CPR) * 8;
  const int c = c0 + cc;
  float ms[8], iv[8], as[8], ab[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ms[j] = a.bmean[c + j]; iv[j] = a.binv[c + j];
    as[j] = a.baff_s[c + j]; ab[j] = a.baff_b[c + j];
  }
  const float al = a.balpha[0];
  // the PReLU alpha partial in fp64: a sum of g * u over every pixel and
  // channel of the tile with heavy cancellation (the 36x52 bottleneck's alpha
  // grad sat at ~8x the fp32 CPU reference's error with fp32 partials)
  float s0[8], s1[8];
  double sa = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) { s0[j] = 0.f; s1[j] = 0.f; }
  // every chunk's t loaded before the first gm store (a store may alias a
  // later load: in program order each chunk paid a memory latency)
  f32x4 tp[NCH][2];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int r = (tid + NT * i) / CPR;
    const long long e = (long long)(p0 + (r < nvalid ? r : 0)) * a.cout + c;
    tp[i][0] = load4<T>(reinterpret_cast<const T *>(a.bt) + e);
    tp[i][1] = load4<T>(reinterpret_cast<const T *>(a.bt) + e + 4);
  }
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int q = tid + NT * i;
    const int r = q / CPR;
    if (r >= nvalid) continue;
    const long long e = (long long)(p0 + r) * a.cout + c;
    const f32x4 g0 = *reinterpret_cast<const f32x4 *>(stg + r * SROW + cc);
    const f32x4 g1 = *reinterpret_cast<const f32x4 *>(stg + r * SROW + cc + 4);
    const f32x4 t0 = tp[i][0];
    const f32x4 t1 = tp[i][1];
    const float g[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
    const float t[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
    float gm[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float u = t[j] * as[j] + ab[j];            // BN output (PReLU input)
      sa += u > 0.f ? 0.0 : (double)(g[j] * u);
      gm[j] = u > 0.f ? g[j] : al * g[j];
      s0[j] += gm[j];
      s1[j] += gm[j] * ((t[j] - ms[j]) * iv[j]);
    }
    store8<T>(reinterpret_cast<T *>(a.y1) + e, f32x4{gm[0], gm[1], gm[2], gm[3]},
              f32x4{gm[4], gm[5], gm[6], gm[7]});
  }
#pragma unroll
  for (int o = CPR; o < 64; o <<= 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s0[j] += __shfl_xor(s0[j], o, 64);
      s1[j] += __shfl_xor(s1[j], o, 64);
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) sa += __shfl_xor(sa, o, 64);
  __syncthreads();                             // stg reads done before red is written
  float *red = stg + BP * SROW;                // [NW][BC][2] floats + [NW] doubles
  const int lane = tid & 63, wv = tid >> 6;
  if (lane < CPR) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wv * BC + cc + j) * 2 + 0] = s0[j];
      red[(wv * BC + cc + j) * 2 + 1] = s1[j];
    }
  }
  double *redd = reinterpret_cast<double *>(red + NW * BC * 2);   // (8-B aligned)
  if (lane == 0) redd[wv] = sa;
  __syncthreads();
  for (int cl = tid; cl < BC; cl += NT) {
    float x = 0.f, y = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      x += red[(q * BC + cl) * 2 + 0];
      y += red[(q * BC + cl) * 2 + 1];
    }
    float *pp = a.bpart + ((long long)pblk * a.cout + c0 + cl) * 3;
    pp[0] = x; pp[1] = y; pp[2] = 0.f;
  }
  if (tid == 0) {
    double x = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) x += redd[q];
    // layout [npblk][cout / 64] (independent of BC): this tile's sum in its
    // first 64-channel slot, zeros in the rest
    float *ap = a.bapart + (long long)pblk * (a.cout / 64) + c0 / 64;
#pragma unroll
    for (int k = 0; k < BC / 64; ++k) ap[k] = k == 0 ? (float)x : 0.f;
  }
}

// Staged epilogue: the fp32 tile sits in LDS as stg[BP][BC + 4] (pre-bias
// accumulators, after a barrier).  Column-wise BN partial statistics from
// LDS, then 8-channel chunks (16-B bf16 / 32-B f32 stores, row-contiguous per
// wave) with bias, accumulate, ReLU, relu-backward mask, column split and the
// convT 2x2 pixel scatter.  NT threads; needs BC | (the column count).
template <typename T, int BC, int BP, int NT, int MODE>
__device__ __forceinline__ void store_staged(const IgemmArgs &a, float *stg, int c0, int p0,
                                             int pblk, int tid) {
  constexpr int SROW = BC + 4;
  const int nvalid = min(BP, a.P - p0);
  if (a.bpart) {
    store_staged_bnbwd<T, BC, BP, NT>(a, stg, c0, p0, pblk, tid, nvalid);
    return;
  }
  if (a.stats) {
    constexpr int TPC = NT / BC;            // threads per channel column
    float *red = stg + BP * SROW;            // [TPC][BC][2]
    const int c = tid % BC, sl = tid / BC;
    // four independent chains (LDS latency, not bandwidth, bounds this loop);
    // fixed combine order -> deterministic
    float x0 = 0.f, y0 = 0.f, x1 = 0.f, y1 = 0.f, x2 = 0.f, y2 = 0.f, x3 = 0.f, y3 = 0.f;
    int r = sl;
    for (; r + 3 * TPC < nvalid; r += 4 * TPC) {
      const float v0 = stg[r * SROW + c], v1 = stg[(r + TPC) * SROW + c];
      const float v2 = stg[(r + 2 * TPC) * SROW + c], v3 = stg[(r + 3 * TPC) * SROW + c];
      x0 += v0; y0 += v0 * v0; x1 += v1; y1 += v1 * v1;
      x2 += v2; y2 += v2 * v2; x3 += v3; y3 += v3 * v3;
    }
    for (; r < nvalid; r += TPC) {
      const float v = stg[r * SROW + c];
      x0 += v; y0 += v * v;
    }
    const float x = (x0 + x1) + (x2 + x3), y = (y0 + y1) + (y2 + y3);
    red[(sl * BC + c) * 2 + 0] = x;
    red[(sl * BC + c) * 2 + 1] = y;
    __syncthreads();
    if (tid < BC) {
      float sx = 0.f, sy = 0.f;
#pragma unroll
      for (int q = 0; q < TPC; ++q) {
        sx += red[(q * BC + tid) * 2 + 0];
        sy += red[(q * BC + tid) * 2 + 1];
      }
      a.stats[((long long)pblk * a.cout + c0 + tid) * 2 + 0] = sx;
      a.stats[((long long)pblk * a.cout + c0 + tid) * 2 + 1] = sy;
    }
  }
  constexpr int CPR = BC / 8;                // 8-channel chunks per pixel row
  constexpr int NCH = BP * CPR / NT;        // chunks per thread
#pragma unroll 2
  for (int i = 0; i < NCH; ++i) {
    const int q = tid + NT * i;
    const int r = q / CPR;
    const int cc = (q - r * CPR) * 8;
    if (r >= nvalid) continue;
    const int p = p0 + r;
    const int c = c0 + cc;
    f32x4 v0 = *reinterpret_cast<const f32x4 *>(stg + r * SROW + cc);
    f32x4 v1 = *reinterpret_cast<const f32x4 *>(stg + r * SROW + cc + 4);
    if (a.bias) {
      v0 += *reinterpret_cast<const f32x4 *>(a.bias + c);
      v1 += *reinterpret_cast<const f32x4 *>(a.bias + c + 4);
    }
    T *dst;
    const T *msk = nullptr;
    if (MODE == RR_CONVT_UP) {
      const int tap = c / a.cout_t;
      const int co = c - tap * a.cout_t;
      const int hw = a.h * a.w;
      const int nn = p / hw;
      const int rem = p - nn * hw;
      const int hh = rem / a.w, ww = rem - (rem / a.w) * a.w;
      const long long op = ((long long)nn * 2 * a.h + 2 * hh + (tap >> 1)) * (2 * a.w) + 2 * ww + (tap & 1);
      dst = reinterpret_cast<T *>(a.y1) + op * a.cout_t + co;
    } else if (a.split > 0 && c >= a.split) {
      dst = reinterpret_cast<T *>(a.y2) + (long long)p * (a.cout - a.split) + (c - a.split);
    } else {
      const int ld = a.split > 0 ? a.split : a.cout;
      dst = reinterpret_cast<T *>(a.y1) + (long long)p * ld + c;
      if (a.has_mask) msk = reinterpret_cast<const T *>(a.mask) + (long long)p * ld + c;
    }
    if (a.accumulate) {
      v0 += load4<T>(dst);
      v1 += load4<T>(dst + 4);
    }
    if ((a.act & 3) == RR_ACT_RELU) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { v0[k] = fmaxf(v0[k], 0.f); v1[k] = fmaxf(v1[k], 0.f); }
    }
    if (msk) {
      const f32x4 m0 = load4<T>(msk), m1 = load4<T>(msk + 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v0[k] = m0[k] > 0.f ? v0[k] : 0.f;
        v1[k] = m1[k] > 0.f ? v1[k] : 0.f;
      }
    }
    store8<T>(dst, v0, v1);
  }
}

}  // namespace
