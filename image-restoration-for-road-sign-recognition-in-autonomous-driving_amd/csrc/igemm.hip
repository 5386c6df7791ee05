// igemm.hip -- implicit-GEMM convolution on CDNA4 MFMA (gfx950).
//
// Replaces the ATen convolution kernels the reference dispatches from
//   nn.Conv2d(k=3, p=1) fwd / dgrad     07:78-96, 14:100-104, VGG16 features
//   nn.Conv2d(k=1) fwd / dgrad          14:111 (shortcut), 07:96 / 14:149 final
//   nn.ConvTranspose2d(k=2, s=2) fwd / dgrad   07:88,92, 14:143-149
//   nn.Linear (h = w = 1)               VGG16 classifier (18:58-61)
//
// GEMM view (NHWC activations, channels contiguous):
//   D[c][p] = sum_k W[c][k] * X[p][k]
//     c : GEMM column = output channel (weights row)       -> MFMA "A" rows
//     p : GEMM row    = output pixel (activation row)      -> MFMA "B" cols
//     k : tap * Cin + ci; X[p][k] gathered from the source pixel of tap
//
// Tile: BC x BP per 256-thread workgroup (4 waves in 2x2), one 128-byte
// k-stage per LDS buffer (bf16: 64 k, f32: 32 k), double buffered.  Both
// operand tiles are filled by global_load_lds_dwordx4 (LDS-DMA): each
// wave-instruction moves 8 rows x 128 B; the per-lane SOURCE address does the
// implicit-GEMM gather (halo taps, concat sources, convT 2x2) and points
// out-of-image rows at a zero page.  The 16-B chunk order inside a row is
// XOR-swizzled on the source side (chunk ^ ((row>>1)&7)) and undone on the
// ds_read_b128 fragment reads, which makes those reads bank-conflict-free.
//
// MFMA: bf16 v_mfma_f32_16x16x32_bf16 (one per 16-B fragment pair);
//       f32  v_mfma_f32_16x16x4_f32 (exact fp32, four per fragment pair).
// Accumulator lane map: pixel = lane&15, channels (lane>>4)*4 .. +3, so each
// lane stores 4 consecutive NHWC channels of one pixel.
//
// Epilogue (fused): per-column partial BN statistics of the pre-bias
// accumulator, + bias, accumulate into the destination, ReLU, multiply by a
// (mask > 0) relu-backward mask, split of the columns over two destinations
// (the grads of a torch.cat's two halves), convT 2x2 pixel scatter.
#include "common.h"

#include <cstdlib>

namespace {

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
  int dbg;            // diagnostics (RR_IGEMM_DBG): bit0 skip epilogue, bit1 K loop x2
};

template <typename T> struct Frag;
template <> struct Frag<bf16_t> {
  using type = bf16x8;
  __device__ __forceinline__ static void mma(f32x4 &acc, const type &a, const type &b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
};
template <> struct Frag<float> {
  using type = f32x4;
  __device__ __forceinline__ static void mma(f32x4 &acc, const type &a, const type &b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], acc, 0, 0, 0);
  }
};

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

constexpr int ROWB = 128;  // bytes of k per row per stage

template <typename T, int BC, int BP, int WC, int MODE>
__global__ __launch_bounds__(256, 2) void igemm_kernel(IgemmArgs a) {
  constexpr int ES = sizeof(T);
  constexpr int BK = ROWB / ES;                 // k elements per stage
  constexpr int WP = 4 / WC;                    // wave grid WC (channels) x WP (pixels)
  constexpr int IA = BC / 32, IB = BP / 32;     // LDS-DMA instructions per wave per stage
  constexpr int STAGE_BYTES = (BC + BP) * ROWB;
  constexpr int MC = BC / WC / 16, MP = BP / WP / 16;   // 16x16 subtiles per wave
  constexpr int SROW = BC + 4;                   // fp32 staging row (floats), padded
  constexpr int STG_BYTES = BP * SROW * 4 + 2 * 256 * 4 * 2;
  constexpr int SMEM = (2 * STAGE_BYTES > STG_BYTES) ? 2 * STAGE_BYTES : STG_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int wc = wv % WC, wp = wv / WC;
  const int cblk = blockIdx.x % a.ncblk;
  const int pblk = blockIdx.x / a.ncblk;
  const int c0 = cblk * BC;
  const int p0 = pblk * BP;

  // ---- per-lane load descriptors (fixed for the whole K loop) -----------
  // instruction i of a wave covers tile rows [8j, 8j+8) with j = wv + 4i;
  // lane -> row 8j + lane/8, physical 16-B chunk lane%8 (loads logical
  // chunk (lane%8) ^ swz(row): the source-side half of the XOR swizzle)
  const int lrow = lane >> 3;
  const int pchunk = lane & 7;
  const char *arow[IA];                 // weight row (+chunk) or nullptr
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int r = 8 * (wv + 4 * i) + lrow;
    const int c = c0 + r;
    arow[i] = (c < a.cout) ? a.wt + ((long long)c * a.K) * ES + ((pchunk ^ swz(r)) << 4) : nullptr;
  }
  // B rows: source pixel base (before the tap offset), validity bits:
  //  bit 0..2: row h+dy in range for dy = -1,0,1; bit 3..5: col w+dx in range
  int bpix[IB], bmask[IB], bchunk[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int r = 8 * (wv + 4 * i) + lrow;
    const int p = p0 + r;
    bchunk[i] = (pchunk ^ swz(r)) << 4;
    if (p < a.P) {
      const int hw = a.h * a.w;
      const int nn = p / hw;
      const int rem = p - nn * hw;
      const int hh = rem / a.w, ww = rem - (rem / a.w) * a.w;
      if (MODE == RR_CONVT_DOWN) {
        bpix[i] = (nn * 2 * a.h + 2 * hh) * (2 * a.w) + 2 * ww;
        bmask[i] = 0x3f;
      } else {
        bpix[i] = p;
        bmask[i] = (hh > 0 ? 1 : 0) | 2 | (hh + 1 < a.h ? 4 : 0) |
                   (ww > 0 ? 8 : 0) | 16 | (ww + 1 < a.w ? 32 : 0);
      }
    } else {
      bpix[i] = 0;
      bmask[i] = 0;
    }
  }

  const int kchunks = a.cin / BK;   // stages per tap
  const int nstage0 = a.taps * kchunks;
  const int nstage = (a.dbg & 2) ? 2 * nstage0 : nstage0;

  auto issue = [&](int s_, int buf) {
    const int s = s_ >= nstage0 ? s_ - nstage0 : s_;
    const int tap = s / kchunks;                 // wave-uniform
    const int ci0 = (s - tap * kchunks) * BK;
    char *sbase = smem + buf * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const char *src = arow[i] ? arow[i] + ((long long)s * BK) * ES : rr_zero_page;
      __builtin_amdgcn_global_load_lds((const void *)src, LDS_PTR(sbase + (wv + 4 * i) * 1024), 16,
                                       0, 0);
    }
    // wave-uniform part of the B address: source, tap offset (pixels), channel
    int toff, vbits;
    if (MODE == RR_CONV3X3) {
      const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
      toff = dy * a.w + dx;
      vbits = (1 << (dy + 1)) | (8 << (dx + 1));
    } else if (MODE == RR_CONVT_DOWN) {
      toff = (tap >> 1) * (2 * a.w) + (tap & 1);
      vbits = 2 | 16;
    } else {
      toff = 0;
      vbits = 2 | 16;
    }
    const bool first = ci0 < a.c1;
    const char *base = first ? a.x1 : a.x2;
    const long long cs = first ? a.c1 : a.c2;
    const long long cofs = (long long)(first ? ci0 : ci0 - a.c1) * ES;
    char *bdst = sbase + BC * ROWB;
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const bool ok = (bmask[i] & vbits) == vbits;
      const char *src = ok ? base + ((long long)(bpix[i] + toff) * cs) * ES + cofs + bchunk[i]
                           : rr_zero_page;
      __builtin_amdgcn_global_load_lds((const void *)src, LDS_PTR(bdst + (wv + 4 * i) * 1024), 16,
                                       0, 0);
    }
  };

  f32x4 acc[MC][MP];
#pragma unroll
  for (int mi = 0; mi < MC; ++mi)
#pragma unroll
    for (int ni = 0; ni < MP; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  using FT = typename Frag<T>::type;
  const int frow = lane & 15;
  const int fq = lane >> 4;

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int s = 0; s < nstage; ++s) {
    const int buf = s & 1;
    if (s + 1 < nstage) issue(s + 1, buf ^ 1);
    const char *sA = smem + buf * STAGE_BYTES;
    const char *sB = sA + BC * ROWB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      FT fa[MC], fb[MP];
#pragma unroll
      for (int mi = 0; mi < MC; ++mi) {
        const int r = wc * (BC / WC) + mi * 16 + frow;
        const int ch = (kk * 4 + fq) ^ swz(r);
        fa[mi] = *reinterpret_cast<const FT *>(sA + r * ROWB + ch * 16);
      }
#pragma unroll
      for (int ni = 0; ni < MP; ++ni) {
        const int r = wp * (BP / WP) + ni * 16 + frow;
        const int ch = (kk * 4 + fq) ^ swz(r);
        fb[ni] = *reinterpret_cast<const FT *>(sB + r * ROWB + ch * 16);
      }
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int ni = 0; ni < MP; ++ni) Frag<T>::mma(acc[mi][ni], fa[mi], fb[ni]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue --------------------------------------------------------
  if (a.dbg & 1) {
    float t = 0.f;
#pragma unroll
    for (int mi = 0; mi < MC; ++mi)
#pragma unroll
      for (int ni = 0; ni < MP; ++ni) t += acc[mi][ni][0];
    if (t == 1234.5f) a.y1[0] = 1;   // keep the accumulators live
    return;
  }
  if (!a.out_nchw && c0 + BC <= a.cout) {
    // ---- staged epilogue: fp32 tile through LDS, column-wise BN stats,
    // ---- 16-B row-contiguous global stores (one 1 KiB run per wave-store)
    float *stg = reinterpret_cast<float *>(smem);
#pragma unroll
    for (int mi = 0; mi < MC; ++mi)
#pragma unroll
      for (int ni = 0; ni < MP; ++ni) {
        const int r = wp * (BP / WP) + ni * 16 + frow;
        const int col = wc * (BC / WC) + mi * 16 + fq * 4;
        *reinterpret_cast<f32x4 *>(stg + r * SROW + col) = acc[mi][ni];
      }
    __syncthreads();
    const int nvalid = min(BP, a.P - p0);
    if (a.stats) {
      constexpr int TPC = 256 / BC;            // threads per channel column
      float *red = stg + BP * SROW;            // [TPC][BC][2]
      const int c = tid % BC, sl = tid / BC;
      float x = 0.f, y = 0.f;
      for (int r = sl; r < nvalid; r += TPC) {
        const float v = stg[r * SROW + c];
        x += v;
        y += v * v;
      }
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
    constexpr int NCH = BP * CPR / 256;        // chunks per thread
#pragma unroll 2
    for (int i = 0; i < NCH; ++i) {
      const int q = tid + 256 * i;
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
      if (a.act == RR_ACT_RELU) {
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
    return;
  }

  float s1[MC][4], s2[MC][4];
#pragma unroll
  for (int mi = 0; mi < MC; ++mi)
#pragma unroll
    for (int i = 0; i < 4; ++i) { s1[mi][i] = 0.f; s2[mi][i] = 0.f; }

#pragma unroll
  for (int ni = 0; ni < MP; ++ni) {
    const int p = p0 + wp * (BP / WP) + ni * 16 + frow;
    if (p >= a.P) continue;
    long long outpix = p;   // convT_up: recomputed per column (depends on tap)
    int nn = 0, hh = 0, ww = 0;
    if (MODE == RR_CONVT_UP) {
      const int hw = a.h * a.w;
      nn = p / hw;
      const int rem = p - nn * hw;
      hh = rem / a.w;
      ww = rem - hh * a.w;
    }
#pragma unroll
    for (int mi = 0; mi < MC; ++mi) {
      const int cb = c0 + wc * (BC / WC) + mi * 16 + fq * 4;
      if (cb >= a.cout) continue;
      f32x4 v = acc[mi][ni];
      if (a.stats) {
#pragma unroll
        for (int i = 0; i < 4; ++i) { s1[mi][i] += v[i]; s2[mi][i] += v[i] * v[i]; }
      }
      if (a.out_nchw) {
        // model-boundary epilogue: fp32 NCHW (16 lanes = 16 consecutive pixels
        // of one channel plane -> 64-B coalesced per register)
        const int hw = a.h * a.w;
        const int nn2 = p / hw, rem = p - nn2 * hw;
        float *yo = reinterpret_cast<float *>(a.y1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = cb + i;
          if (c >= a.cout) break;
          float x = v[i] + (a.bias ? a.bias[c] : 0.f);
          const long long o = ((long long)nn2 * a.cout + c) * hw + rem;
          if (a.accumulate) x += yo[o];
          if (a.act == RR_ACT_RELU) x = fmaxf(x, 0.f);
          yo[o] = x;
        }
        continue;
      }
      T *dst;
      const T *msk = nullptr;
      int cc = cb;
      if (MODE == RR_CONVT_UP) {
        const int tap = cb / a.cout_t;
        cc = cb - tap * a.cout_t;
        outpix = ((long long)nn * 2 * a.h + 2 * hh + (tap >> 1)) * (2 * a.w) + 2 * ww + (tap & 1);
        dst = reinterpret_cast<T *>(a.y1) + outpix * a.cout_t + cc;
      } else if (a.split > 0 && cb >= a.split) {
        cc = cb - a.split;
        dst = reinterpret_cast<T *>(a.y2) + outpix * (a.cout - a.split) + cc;
      } else {
        const int ld = a.split > 0 ? a.split : a.cout;
        dst = reinterpret_cast<T *>(a.y1) + outpix * ld + cb;
        if (a.has_mask) msk = reinterpret_cast<const T *>(a.mask) + outpix * ld + cb;
      }
      const bool full = (cb + 3 < a.cout);
      if (full) {
        if (a.bias) v += *reinterpret_cast<const f32x4 *>(a.bias + cb);
        if (a.accumulate) v += load4<T>(dst);
        if (a.act == RR_ACT_RELU) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
        }
        if (msk) {
          const f32x4 m = load4<T>(msk);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = m[i] > 0.f ? v[i] : 0.f;
        }
        store4<T>(dst, v);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (cb + i >= a.cout) break;
          float x = v[i];
          if (a.bias) x += a.bias[cb + i];
          if (a.accumulate) x += Elt<T>::load(dst, i);
          if (a.act == RR_ACT_RELU) x = fmaxf(x, 0.f);
          if (msk && !(Elt<T>::load(msk, i) > 0.f)) x = 0.f;
          Elt<T>::store(dst, i, x);
        }
      }
    }
  }

  if (a.stats) {
    // reduce over the 16 pixel lanes that share (lane>>4), then over wp.
#pragma unroll
    for (int mi = 0; mi < MC; ++mi)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float x = s1[mi][i], y = s2[mi][i];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          x += __shfl_xor(x, o, 64);
          y += __shfl_xor(y, o, 64);
        }
        s1[mi][i] = x; s2[mi][i] = y;
      }
    float *red = reinterpret_cast<float *>(smem);   // [WP][BC][2]
    // (the K loop ended with a barrier; smem is free)
    if (frow == 0) {
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int cl = wc * (BC / WC) + mi * 16 + fq * 4 + i;
          red[(wp * BC + cl) * 2 + 0] = s1[mi][i];
          red[(wp * BC + cl) * 2 + 1] = s2[mi][i];
        }
    }
    __syncthreads();
    for (int cl = tid; cl < BC; cl += 256) {
      const int c = c0 + cl;
      if (c < a.cout) {
        float x = 0.f, y = 0.f;
#pragma unroll
        for (int q = 0; q < WP; ++q) {
          x += red[(q * BC + cl) * 2 + 0];
          y += red[(q * BC + cl) * 2 + 1];
        }
        a.stats[((long long)pblk * a.cout + c) * 2 + 0] = x;
        a.stats[((long long)pblk * a.cout + c) * 2 + 1] = y;
      }
    }
  }
}

template <typename T, int BC, int BP, int WC>
int launch_mode(const rr_igemm_desc *d, IgemmArgs &a, hipStream_t st) {
  a.ncblk = (a.cout + BC - 1) / BC;
  const long long npblk = ((long long)a.P + BP - 1) / BP;
  const long long nblk = npblk * a.ncblk;
  if (nblk > 0x7fffffffLL) return RR_EUNSUPPORTED;
  dim3 grid((unsigned)nblk), block(256);
  switch (d->mode) {
    case RR_CONV3X3: hipLaunchKernelGGL((igemm_kernel<T, BC, BP, WC, RR_CONV3X3>), grid, block, 0, st, a); break;
    case RR_CONV1X1: hipLaunchKernelGGL((igemm_kernel<T, BC, BP, WC, RR_CONV1X1>), grid, block, 0, st, a); break;
    case RR_CONVT_UP: hipLaunchKernelGGL((igemm_kernel<T, BC, BP, WC, RR_CONVT_UP>), grid, block, 0, st, a); break;
    case RR_CONVT_DOWN: hipLaunchKernelGGL((igemm_kernel<T, BC, BP, WC, RR_CONVT_DOWN>), grid, block, 0, st, a); break;
    default: return RR_EINVAL;
  }
  RR_CHECK_LAUNCH();
  return RR_OK;
}

// tile choice: (BC, BP) -- the stat-partial row block is BP pixels
struct Tile { int bc, bp; };

Tile pick_tile(const rr_igemm_desc *d) {
  const long long P = (long long)d->n * d->h * d->w;
  const bool split_ok128 = d->out_split == 0 || d->out_split % 128 == 0;
  if (d->c_out % 128 == 0 && split_ok128 && ((P + 127) / 128) * (d->c_out / 128) >= 512)
    return {128, 128};
  if (d->c_out <= 64 && (P + 255) / 256 >= 512) return {64, 256};
  return {64, 128};
}

template <typename T>
int dispatch(const rr_igemm_desc *d, IgemmArgs &a, hipStream_t st) {
  const Tile t = pick_tile(d);
  if (t.bc == 128) return launch_mode<T, 128, 128, 2>(d, a, st);
  if (t.bp == 256) return launch_mode<T, 64, 256, 1>(d, a, st);
  return launch_mode<T, 64, 128, 2>(d, a, st);
}

}  // namespace

extern "C" int rr_igemm_stat_blocks(const rr_igemm_desc *d) {
  if (!d) return RR_EINVAL;
  const long long P = (long long)d->n * d->h * d->w;
  const int bp = pick_tile(d).bp;
  return (int)((P + bp - 1) / bp);
}

extern "C" int rr_igemm(const rr_igemm_desc *d, const void *x1, const void *x2,
                        const void *w, const float *bias, void *y1, void *y2,
                        const void *mask, float *stats_partial, rr_stream stream) {
  if (!d || !x1 || !w || !y1) return RR_EINVAL;
  if (d->dtype != RR_F32 && d->dtype != RR_BF16) return RR_EINVAL;
  const int bk = d->dtype == RR_F32 ? 32 : 64;
  if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c_out <= 0 || d->c_in1 <= 0) return RR_EINVAL;
  if (d->c_in1 % bk || d->c_in2 % bk) return RR_EUNSUPPORTED;
  if (d->c_in2 > 0 && !x2) return RR_EINVAL;
  if (d->out_split > 0 && (!y2 || d->out_split % 64 || d->out_split >= d->c_out)) return RR_EUNSUPPORTED;
  if (d->mode == RR_CONVT_UP && (d->c_out % 4 || (d->c_out / 4) % 64 || d->out_split || d->want_stats))
    return RR_EUNSUPPORTED;
  if (d->has_mask && (!mask || d->out_split)) return RR_EINVAL;
  if (d->out_nchw && (d->out_split || d->has_mask || d->mode == RR_CONVT_UP)) return RR_EINVAL;
  if (d->want_stats && !stats_partial) return RR_EINVAL;
  const long long P = (long long)d->n * d->h * d->w;
  if (P > 0x7fffffffLL / 4) return RR_EUNSUPPORTED;
  IgemmArgs a;
  a.x1 = (const char *)x1; a.x2 = (const char *)x2; a.wt = (const char *)w;
  a.bias = bias; a.y1 = (char *)y1; a.y2 = (char *)y2; a.mask = (const char *)mask;
  a.stats = d->want_stats ? stats_partial : nullptr;
  a.n = d->n; a.h = d->h; a.w = d->w;
  a.c1 = d->c_in1; a.c2 = d->c_in2; a.cin = d->c_in1 + d->c_in2;
  a.cout = d->c_out; a.split = d->out_split;
  a.act = d->act; a.accumulate = d->accumulate; a.has_mask = d->has_mask;
  a.taps = d->mode == RR_CONV3X3 ? 9 : (d->mode == RR_CONVT_DOWN ? 4 : 1);
  a.K = a.taps * a.cin;
  a.P = (int)P;
  a.cout_t = d->mode == RR_CONVT_UP ? d->c_out / 4 : d->c_out;
  a.out_nchw = d->out_nchw;
  static const int dbg_env = [] { const char *e = getenv("RR_IGEMM_DBG"); return e ? atoi(e) : 0; }();
  a.dbg = dbg_env;
  a.ncblk = 1;
  hipStream_t st = (hipStream_t)stream;
  if (d->dtype == RR_BF16) return dispatch<bf16_t>(d, a, st);
  return dispatch<float>(d, a, st);
}
