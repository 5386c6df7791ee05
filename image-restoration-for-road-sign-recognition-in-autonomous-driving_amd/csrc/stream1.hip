// stream1.hip -- wave-streaming bf16 GEMM for the convolutions with no
// spatial taps to share: nn.Conv2d(k=1) fwd / dgrad (ResidualBlock shortcut
// 14:109-112, ResUNet final conv 14:149), nn.ConvTranspose2d(k=2, s=2) fwd
// (14:137-147 up3/up2/up1) and its dgrad.  Called from rr_igemm (igemm.hip)
// for the large-pixel-count shapes; not part of the C ABI.
//
// Why a separate kernel.  These GEMMs have K = 64..384: one or a few 64-deep
// k-stages, so a tiled kernel that loads a tile, waits, computes and stores
// is a chain of HBM latencies with nothing to overlap them (the tiled igemm
// ran them at 2-4 TB/s).  They are HBM-bound (K / 2 FLOP per byte), so the
// goal is a continuous stream:
//   * every wave owns a slice of 16 MC GEMM columns with ALL of K -- its MFMA
//     A fragments (MC x KB x 16 B per lane) stay in registers for the kernel;
//   * it walks 16-pixel blocks b = gw, gw + NWT, ... (all waves of a slice
//     together sweep a contiguous window of memory) and loads each block's
//     B fragments straight from global memory into registers (16 B per lane:
//     8 channels of one pixel; two lane rows cover a 128-B line), D blocks
//     ahead of the MFMAs -- no LDS, no workgroup barrier in the loop;
//   * the epilogue works in registers: BN statistics of the pre-bias
//     accumulators kept across all of the wave's blocks (one reduction at
//     the end, per-workgroup partial rows), a permlane16 swap of each pair of
//     16-column fragments so a lane holds 8 consecutive columns of one pixel,
//     then bias / accumulate / ReLU / relu-mask and one 16-B store per lane
//     (column split of a concat grad, convT 2x2 pixel scatter by column).
// The model-boundary final conv (c_out <= 16, fp32 NCHW output) stores from
// the accumulator layout: 16 lanes = 16 consecutive pixels of one plane.
#include "common.h"
#include "stream1.h"

#include <cstdio>
#include <cstdlib>

namespace {

enum : int { G_BIAS = 1, G_RELU = 2 };

constexpr int S1_NW = 4;   // waves per workgroup

__device__ __forceinline__ f32x4 unpack_lo(uint4 v) {
  return f32x4{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
               __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u)};
}
__device__ __forceinline__ f32x4 unpack_hi(uint4 v) {
  return f32x4{__uint_as_float(v.z << 16), __uint_as_float(v.z & 0xffff0000u),
               __uint_as_float(v.w << 16), __uint_as_float(v.w & 0xffff0000u)};
}
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return (uint32_t)f32_to_bf16(a) | ((uint32_t)f32_to_bf16(b) << 16);
}

// MC: 16-column fragments per wave; KB: 32-deep k fragments (K = 32 KB).
// STATS: per-column sums of the pre-bias accumulator (registers held over
// the loop, so a template flag).  MODE: RR_CONV1X1 / RR_CONVT_UP /
// RR_CONVT_DOWN.  NCHW: the fp32 NCHW boundary store.  EOP: epilogue
// operand per output element -- E_ACC the destination's previous value,
// E_MASK the relu-backward mask -- loaded WITH the block's B fragments, so
// the wait for a block covers them (an operand loaded in the epilogue would
// make the wave wait for every prefetch older than it: vmcnt is in order).
// D: blocks in flight per wave.  The bias sits in LDS (lgkmcnt, not vmcnt).
enum : int { E_NONE = 0, E_ACC = 1, E_MASK = 2 };

template <int MC, int KB, bool STATS, int MODE, bool NCHW, int EOP>
__global__ __launch_bounds__(256, 2) void stream1_kernel(S1Args a) {
  // (KB = 12 with the statistics registers keeps 1 block in flight: 2 spill
  // 54 VGPRs)
  constexpr int D0 = KB <= 2 ? 4 : (KB <= 4 ? 3 : (KB <= 8 || !STATS ? 2 : 1));
  constexpr int D = (EOP != E_NONE && MC >= 8) ? 2 : D0;
  constexpr int CW = 16 * MC;
  constexpr int NQ = MC / 2 > 0 ? MC / 2 : 1;
  const int lane = threadIdx.x & 63;
  // wave-uniform in SGPRs: the block loop's bounds and the epilogue's flag
  // tests then branch on scalars instead of exec masks
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int flags = __builtin_amdgcn_readfirstlane(a.flags);
  const bool fbias = (flags & G_BIAS) != 0, frelu = (flags & G_RELU) != 0;
  const int g = blockIdx.x % a.G, slice = blockIdx.x / a.G;
  const int gw = g * S1_NW + wv;                // wave within the slice
  const int NWT = a.G * S1_NW;
  const int frow = lane & 15, fq = lane >> 4;
  const int cbase = slice * CW;                 // first GEMM column of the wave
  const int nblk = a.P >> 4;

  __shared__ __attribute__((aligned(16))) float sbias[CW];
  for (int c = threadIdx.x; c < CW; c += 256)
    sbias[c] = fbias && cbase + c < a.cout ? a.bias[cbase + c] : 0.f;

  // ---- A fragments: GEMM column cbase + mi*16 + frow, k = kb*32 + fq*8 ----
  bf16x8 wr[MC][KB];
#pragma unroll
  for (int mi = 0; mi < MC; ++mi) {
    const int c = cbase + mi * 16 + frow;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      bf16x8 v = {};
      if (c < a.cout) v = *reinterpret_cast<const bf16x8 *>(a.wt + ((long long)c * a.K + kb * 32 + fq * 8) * 2);
      wr[mi][kb] = v;
    }
  }
  __syncthreads();                              // sbias

  // fine-grid pixel (2y, 2x) of coarse pixel p (convT up / down)
  auto fine_of = [&](int p) __attribute__((always_inline)) {
    const int n = (int)fdiv((uint32_t)p, a.fd_hw), rem = p - n * a.hw;
    const int y = (int)fdiv((uint32_t)rem, a.fd_w), x = rem - y * a.w;
    return (long long)(n * 2 * a.h + 2 * y) * 2 * a.w + 2 * x;
  };
  // the lane's first column of widened pair q (see the epilogue)
  auto col_of = [&](int q) __attribute__((always_inline)) {
    return cbase + (2 * q + (fq & 1)) * 16 + (fq >> 1) * 8;
  };
  // output byte offset of the lane's 8 columns c .. c + 7 of pixel p (NHWC
  // bf16) and its destination.  The 32 columns of a widened pair q start at
  // cq = cbase + 32 q; split and the convT tap width are multiples of 32
  // (planner), so the destination and the tap are wave-uniform per pair.
  char *const y1 = a.y1, *const y2 = a.y2;
  const char *const mask = a.mask;
  auto out_off = [&](int p, int q, long long fine, char *&base) __attribute__((always_inline)) {
    const int cq = cbase + 32 * q;
    const int c = col_of(q);
    if constexpr (MODE == RR_CONVT_UP) {
      const int tap = cq / a.cout_t, co = c - tap * a.cout_t;
      base = y1;
      return ((fine + (tap >> 1) * 2 * a.w + (tap & 1)) * a.cout_t + co) * 2;
    } else {
      const bool second = a.split > 0 && cq >= a.split;
      base = second ? y2 : y1;
      return second ? ((long long)p * (a.cout - a.split) + (c - a.split)) * 2
                    : ((long long)p * (a.split > 0 ? a.split : a.cout) + c) * 2;
    }
  };
  struct Blk {
    uint4 b[KB];
    uint4 e[EOP != E_NONE ? NQ : 1];
  };
  // ---- block b's B fragments (pixel b*16 + frow, k = kb*32 + fq*8) and
  // ---- epilogue operands
  auto load_blk = [&](int b, Blk &bk) __attribute__((always_inline)) {
    const int p = b * 16 + frow;
    long long fine = 0;
    if constexpr (MODE == RR_CONVT_DOWN) fine = fine_of(p);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const char *src = a.ksrc[kb] ? a.x2 : a.x1;
      const long long cs = a.ksrc[kb] ? a.c2 : a.c1;
      long long pix = p;
      if constexpr (MODE == RR_CONVT_DOWN) pix = fine + a.ktap[kb];
      bk.b[kb] = *reinterpret_cast<const uint4 *>(src + (pix * cs + a.kch[kb] + fq * 8) * 2);
    }
    if constexpr (EOP != E_NONE) {
      long long ufine = 0;
      if constexpr (MODE == RR_CONVT_UP) ufine = fine_of(p);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        char *base;
        const long long o = out_off(p, q, ufine, base);
        bk.e[q] = *reinterpret_cast<const uint4 *>((EOP == E_MASK ? mask : base) + o);
      }
    }
  };

  f32x4 r0[STATS ? MC : 1], r1[STATS ? MC : 1];
#pragma unroll
  for (int mi = 0; mi < (STATS ? MC : 1); ++mi) { r0[mi] = f32x4{0.f, 0.f, 0.f, 0.f}; r1[mi] = r0[mi]; }

  auto epilogue = [&](const f32x4 (&acc)[MC], const Blk &bk, int b) __attribute__((always_inline)) {
    const int p = b * 16 + frow;
    if constexpr (STATS) {
#pragma unroll
      for (int mi = 0; mi < MC; ++mi) { r0[mi] += acc[mi]; r1[mi] += acc[mi] * acc[mi]; }
    }
    if constexpr (NCHW) {
      // fp32 NCHW, columns < c_out (<= 16: MC = 1): 16 lanes = 16 pixels of one plane
      const int n = p / a.hw, rem = p - (p / a.hw) * a.hw;
      float *yo = reinterpret_cast<float *>(a.y1);
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = cbase + mi * 16 + fq * 4 + j;
          if (c < a.cout) {
            float v = acc[mi][j] + sbias[c - cbase];
            if (frelu) v = fmaxf(v, 0.f);
            yo[((long long)n * a.cout + c) * a.hw + rem] = v;
          }
        }
      return;
    }
    long long fine = 0;
    if constexpr (MODE == RR_CONVT_UP) fine = fine_of(p);
#pragma unroll
    for (int q = 0; q < MC / 2; ++q) {
      // swap the odd lane rows of fragment 2q with the even rows of 2q + 1:
      // lane row r then holds 8 consecutive columns of its pixel,
      // (2q + (r & 1)) * 16 + (r >> 1) * 8 .. + 7
      float lo[4], hi[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * q][j]),
                                                        __float_as_uint(acc[2 * q + 1][j]), false, false);
        lo[j] = __uint_as_float(s[0]);
        hi[j] = __uint_as_float(s[1]);
      }
      const int c = col_of(q);
      f32x4 v0 = f32x4{lo[0], lo[1], lo[2], lo[3]}, v1 = f32x4{hi[0], hi[1], hi[2], hi[3]};
      if (fbias) {
        v0 += *reinterpret_cast<const f32x4 *>(sbias + (c - cbase));
        v1 += *reinterpret_cast<const f32x4 *>(sbias + (c - cbase) + 4);
      }
      if constexpr (EOP == E_ACC) {
        v0 += unpack_lo(bk.e[q]);
        v1 += unpack_hi(bk.e[q]);
      }
      if (frelu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { v0[j] = fmaxf(v0[j], 0.f); v1[j] = fmaxf(v1[j], 0.f); }
      }
      if constexpr (EOP == E_MASK) {
        const f32x4 m0 = unpack_lo(bk.e[q]), m1 = unpack_hi(bk.e[q]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v0[j] = m0[j] > 0.f ? v0[j] : 0.f;
          v1[j] = m1[j] > 0.f ? v1[j] : 0.f;
        }
      }
      char *base;
      const long long o = out_off(p, q, fine, base);
      *reinterpret_cast<uint4 *>(base + o) =
          make_uint4(pk2(v0[0], v0[1]), pk2(v0[2], v0[3]), pk2(v1[0], v1[1]), pk2(v1[2], v1[3]));
    }
  };
  auto compute = [&](const Blk &bk, f32x4 (&acc)[MC]) __attribute__((always_inline)) {
#pragma unroll
    for (int mi = 0; mi < MC; ++mi) acc[mi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
        acc[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mi][kb], __builtin_bit_cast(bf16x8, bk.b[kb]),
                                                          acc[mi], 0, 0, 0);
  };

  // ---- the stream: D blocks in flight per wave.  Full rounds carry no
  // ---- conditional memory op (the compiler's counted waits stay partial);
  // ---- the last, partial round only computes and stores.
  const int niter = gw < nblk ? (nblk - gw + NWT - 1) / NWT : 0;
  const int nfull = niter / D;
  auto blk = [&](int i) __attribute__((always_inline)) {
    const int b = gw + i * NWT;
    return b < nblk ? b : nblk - 1;                // clamped: loads stay unconditional
  };
  Blk ring[D];
#pragma unroll
  for (int j = 0; j < D; ++j) load_blk(blk(j), ring[j]);
  for (int r = 0; r < nfull; ++r) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      f32x4 acc[MC];
      compute(ring[j], acc);
      const Blk cur = ring[j];                   // epilogue operands of this block
      load_blk(blk((r + 1) * D + j), ring[j]);
      epilogue(acc, cur, gw + (r * D + j) * NWT);
    }
  }
#pragma unroll
  for (int j = 0; j < D; ++j) {
    if (nfull * D + j < niter) {
      f32x4 acc[MC];
      compute(ring[j], acc);
      epilogue(acc, ring[j], gw + (nfull * D + j) * NWT);
    }
  }

  // ---- per-workgroup statistics partials: lanes of a column -> waves ----
  if constexpr (STATS) {
    __shared__ float red[S1_NW][CW][2];
#pragma unroll
    for (int mi = 0; mi < MC; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        {
          r0[mi][j] = row16_sum(r0[mi][j]);
          r1[mi][j] = row16_sum(r1[mi][j]);
        }
    if (frow == 0) {
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          red[wv][mi * 16 + fq * 4 + j][0] = r0[mi][j];
          red[wv][mi * 16 + fq * 4 + j][1] = r1[mi][j];
        }
    }
    __syncthreads();
    for (int cl = threadIdx.x; cl < CW; cl += 256) {
      const int c = cbase + cl;
      if (c < a.cout) {
        float x = 0.f, y = 0.f;
#pragma unroll
        for (int w = 0; w < S1_NW; ++w) { x += red[w][cl][0]; y += red[w][cl][1]; }
        a.stats[((long long)g * a.cout + c) * 2 + 0] = x;
        a.stats[((long long)g * a.cout + c) * 2 + 1] = y;
      }
    }
  }
}

// the instantiated kernels: (MC, KB, STATS, MODE, NCHW, EOP)
#define S1_LIST(X)                                                                                 \
  X(4, 2, true, RR_CONV1X1, false, E_NONE) X(4, 4, true, RR_CONV1X1, false, E_NONE)                \
  X(2, 2, true, RR_CONV1X1, false, E_NONE) X(2, 4, true, RR_CONV1X1, false, E_NONE)                \
  X(2, 8, true, RR_CONV1X1, false, E_NONE)                                                         \
  X(2, 12, true, RR_CONV1X1, false, E_NONE)                                                        \
  X(1, 2, false, RR_CONV1X1, true, E_NONE)                                                         \
  X(8, 2, false, RR_CONV1X1, false, E_NONE) X(4, 2, false, RR_CONV1X1, false, E_NONE)              \
  X(4, 4, false, RR_CONV1X1, false, E_NONE) X(2, 4, false, RR_CONV1X1, false, E_NONE)              \
  X(2, 6, false, RR_CONV1X1, false, E_NONE) X(2, 8, false, RR_CONV1X1, false, E_NONE)              \
  X(2, 12, false, RR_CONV1X1, false, E_NONE)                                                       \
  X(8, 2, false, RR_CONV1X1, false, E_ACC) X(4, 2, false, RR_CONV1X1, false, E_ACC)                \
  X(4, 4, false, RR_CONV1X1, false, E_ACC) X(2, 8, false, RR_CONV1X1, false, E_ACC)                \
  X(4, 4, false, RR_CONV1X1, false, E_MASK)                                                        \
  X(8, 2, false, RR_CONVT_UP, false, E_NONE) X(4, 2, false, RR_CONVT_UP, false, E_NONE)            \
  X(4, 4, false, RR_CONVT_UP, false, E_NONE) X(2, 4, false, RR_CONVT_UP, false, E_NONE)            \
  X(2, 8, false, RR_CONVT_UP, false, E_NONE)

constexpr int s1_key(int mc, int kb, bool stats, int mode, bool nchw, int eop) {
  return ((((mc * 16 + kb) * 2 + (stats ? 1 : 0)) * 4 + mode) * 2 + (nchw ? 1 : 0)) * 3 + eop;
}

bool s1_has(int key) {
#define S1_HAS(mc, kb, st, md, nc, eo) if (key == s1_key(mc, kb, st, md, nc, eo)) return true;
  S1_LIST(S1_HAS)
#undef S1_HAS
  return false;
}

// MC of a call: A fragments <= 64-96 VGPRs per lane, fewer with the
// statistics registers (no spills, 2 waves per SIMD); MC even (pairs of
// fragments are widened together) except the 1-fragment NCHW boundary conv
int pick_mc(int kb, int ncol, bool stats, bool nchw) {
  if (nchw) return ncol <= 16 ? 1 : 0;
  int mc = stats ? (kb <= 4 ? 4 : 2) : (kb <= 2 ? 8 : (kb <= 4 ? 4 : 2));
  while (mc > 2 && ncol % (16 * mc)) mc >>= 1;
  return ncol % (16 * mc) == 0 ? mc : 0;
}

bool kb_ok(int kb) { return kb == 2 || kb == 4 || kb == 6 || kb == 8 || kb == 12; }

int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

}  // namespace

int stream1_plan(const rr_igemm_desc *d, S1Plan *pl) {
  // RR_PATH stream1=0: the tiled igemm instead; stream1_minp=N: stream from
  // N pixels (the tests' small shapes; default 131072, measured, r5ze)
  if (!rr_path("stream1", 1)) return 0;
  if (!d || d->dtype != RR_BF16) return 0;
  const int mode = d->mode;
  if (mode != RR_CONV1X1 && mode != RR_CONVT_UP && mode != RR_CONVT_DOWN) return 0;
  const long long P = (long long)d->n * d->h * d->w;
  const long long minp = rr_path("stream1_minp", 131072);
  if (P < minp || P % 16 || P * 16 > 0x7fffffffLL) return 0;
  const int cin = d->c_in1 + d->c_in2;
  const int taps = mode == RR_CONVT_DOWN ? 4 : 1;
  if (d->c_in1 % 32 || d->c_in2 % 32) return 0;
  const int kb = taps * cin / 32;
  if (!kb_ok(kb)) return 0;
  if (d->out_nchw && (mode != RR_CONV1X1 || d->has_mask || d->out_split)) return 0;
  if (d->has_mask && d->out_split) return 0;
  if (mode != RR_CONV1X1 && d->c_in2) return 0;
  if (mode != RR_CONV1X1 && d->want_stats) return 0;
  if (mode != RR_CONV1X1 && mode != RR_CONVT_DOWN && d->has_mask) return 0;
  if (mode == RR_CONVT_UP && (d->c_out % 4 || (d->c_out / 4) % 8)) return 0;
  if (d->out_split && d->out_split % 32) return 0;
  if (mode == RR_CONVT_UP && (d->c_out / 4) % 32) return 0;
  if (d->accumulate && d->has_mask) return 0;
  if (d->out_nchw && d->accumulate) return 0;
  const int eop = d->accumulate ? E_ACC : (d->has_mask ? E_MASK : E_NONE);
  const int mc = pick_mc(kb, d->c_out, d->want_stats != 0, d->out_nchw != 0);
  if (!mc || !s1_has(s1_key(mc, kb, d->want_stats != 0, mode, d->out_nchw != 0, eop))) return 0;
  const int nslice = (d->c_out + 16 * mc - 1) / (16 * mc);
  int G = 512 / nslice;
  G = G >= 8 ? G & ~7 : 1;                        // slices of one pixel window share an XCD
  pl->mc = mc;
  pl->kb = kb;
  pl->key = s1_key(mc, kb, d->want_stats != 0, mode, d->out_nchw != 0, eop);
  pl->nslice = nslice;
  pl->G = G;
  return G;
}

int stream1_launch(const rr_igemm_desc *d, const S1Plan &pl, S1Args a, hipStream_t stream) {
  const int cin = d->c_in1 + d->c_in2;
  a.mode = d->mode;
  a.P = d->n * d->h * d->w;
  a.h = d->h; a.w = d->w;
  a.hw = d->h * d->w;
  a.lw = ilog2(d->w) < 0 ? 0 : ilog2(d->w);
  a.lhw = ilog2(d->h * d->w) < 0 ? 0 : ilog2(d->h * d->w);
  a.fd_hw = make_fastdiv((uint32_t)(d->h * d->w));
  a.fd_w = make_fastdiv((uint32_t)d->w);
  a.c1 = d->c_in1; a.c2 = d->c_in2;
  a.cout = d->c_out;
  a.cout_t = d->mode == RR_CONVT_UP ? d->c_out / 4 : d->c_out;
  a.split = d->out_split;
  a.K = pl.kb * 32;
  a.G = pl.G;
  a.flags = (d->has_bias ? G_BIAS : 0) | (d->act == RR_ACT_RELU ? G_RELU : 0);
  for (int kb = 0; kb < pl.kb; ++kb) {
    const int k = kb * 32;
    const int tap = d->mode == RR_CONVT_DOWN ? k / cin : 0;
    const int ci = k - tap * cin;
    a.ksrc[kb] = ci >= d->c_in1 ? 1 : 0;
    a.kch[kb] = ci >= d->c_in1 ? ci - d->c_in1 : ci;
    // fine-grid pixel offset of the tap (convT down: x1 on the (2h, 2w) grid)
    a.ktap[kb] = (tap >> 1) * 2 * d->w + (tap & 1);
  }
  const int grid = pl.G * pl.nslice;
#define S1_GO(mc, kb, st, md, nc, eo)                                                                  \
  if (pl.key == s1_key(mc, kb, st, md, nc, eo)) {                                                      \
    hipLaunchKernelGGL((stream1_kernel<mc, kb, st, md, nc, eo>), dim3(grid), dim3(256), 0, stream, a); \
    RR_CHECK_LAUNCH();                                                                                 \
    return RR_OK;                                                                                      \
  }
  S1_LIST(S1_GO)
#undef S1_GO
  return RR_EUNSUPPORTED;
}

const char *stream1_name(const S1Plan &pl) {
  static const char *names[9][17] = {};
  static char buf[9][17][32];
  if (pl.mc < 1 || pl.mc > 8 || pl.kb < 1 || pl.kb > 16) return "stream1_kernel<?>";
  if (!names[pl.mc][pl.kb]) {
    snprintf(buf[pl.mc][pl.kb], sizeof buf[0][0], "stream1_kernel<%d,%d>", pl.mc, pl.kb);
    names[pl.mc][pl.kb] = buf[pl.mc][pl.kb];
  }
  return names[pl.mc][pl.kb];
}
