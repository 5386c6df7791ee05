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
#include "stream3.h"
#include "stream1.h"
#include "igemm_epi.h"
#include "conv3r.h"

#include <cstdlib>
#include <type_traits>

namespace {

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
  constexpr int STG_BYTES = BP * SROW * 4 + 2 * 256 * 4 * 2 + 256;
  constexpr int SMEM = (2 * STAGE_BYTES > STG_BYTES) ? 2 * STAGE_BYTES : STG_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int wc = wv % WC, wp = wv / WC;
  // XCD-aware tile order, as in igemm3_halo_kernel (a.xcd)
  int tile = blockIdx.x;
  if (a.xcd) {
    const int per = (int)gridDim.x / 8;
    if ((int)blockIdx.x < per * 8) tile = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
  }
  const int cblk = tile % a.ncblk;
  const int pblk = tile / a.ncblk;
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
  const int nstage = nstage0;

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
    store_staged<T, BC, BP, 256, MODE>(a, stg, c0, p0, pblk, tid);
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
        s1[mi][i] = row16_sum(s1[mi][i]);
        s2[mi][i] = row16_sum(s2[mi][i]);
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

// ---------------------------------------------------------------------------
// 3x3 bf16 conv (fwd or dgrad) with an LDS halo.  A tile is BP = 256 output
// pixels = R = 256/W whole image rows (or R/H whole images when R > H) x BC
// output channels, 512 threads (8 waves, wave tile 64 ch x 256/WP px).  Per
// 64-channel K chunk the zero-padded input halo -- (Hs+2) x (W+2) rows per
// image, Hs = min(R, H) -- is staged ONCE and serves all 9 taps; the weights
// stream per (chunk, tap).  So the activation is read ~1.3x instead of 9x.
//
// LDS image ("k-planes"): plane j (16-B channel chunk j of the 64) holds the
// rows contiguously, 16 B per row.  A ds_read_b128 16-lane group reads rows
// {0-3,12-15} at chunk q and rows {4-11} at chunk q+1 (MFMA fragment map);
// with plane size = 0 mod 256 B those 16 rows hit 16 distinct 16-B bank
// slots for ANY base row, so every tap's shifted read is conflict-free and
// its address is the lane's base + tap * 16 B.  Fills are register-staged:
// piece idx -> chunk (idx >> 3) & 7, row 8 * (idx >> 6) + (idx & 7): a wave
// instruction reads 8 full 128-B lines and writes 8 x 128 contiguous bytes.
//
// Pipeline: one barrier per (chunk, tap) stage; weights prefetched 2 stages
// ahead in registers, the next chunk's halo loaded at tap 0 and written at
// tap 8.
template <int W, int BP, int NT = 2 * BP> struct HaloGeom {
  static constexpr int R = BP / W;
  // worst case over H >= 8 with H | R or R | H: R/Hs images of (Hs+2) rows
  static constexpr int HMAX = (R <= 8 ? (R + 2) : (R / 8) * 10) * (W + 2);
  static constexpr int PLANE = ((HMAX * 16 + 255) / 256) * 256;
  static constexpr int HBYTES = 8 * PLANE;
  static constexpr int LH = (HMAX * 8 + NT - 1) / NT;             // pieces per thread
};

// BC = 64 keeps ONE halo buffer (the next chunk's halo is written after an
// extra barrier at tap 8), so LDS <= 78 KB and VGPRs <= 128: 2 workgroups
// per CU, one tile's prologue / epilogue overlapping the other's MFMA loop.
// BC = 128 double-buffers the halo, 1 workgroup per CU.
// BP = 128 (256 threads, ~51 KB LDS at BC = 64): 3 workgroups per CU.
template <int BC, int BP, int NT = 2 * BP> struct HaloCfg {
  static constexpr int HB = BC <= 64 ? 1 : 2;
  static constexpr int OCC = NT == BP ? 2 : BP == 128 ? (BC <= 64 ? 3 : 2) : (BC <= 64 ? 4 : 2);   // min waves / SIMD
};

template <int BC, int W, int MODE, int BP, int NT = 2 * BP>
__global__ __launch_bounds__(NT, (HaloCfg<BC, BP, NT>::OCC)) void igemm3_halo_kernel(IgemmArgs a) {
  using T = bf16_t;
  using G = HaloGeom<W, BP, NT>;
  constexpr int HB = HaloCfg<BC, BP, NT>::HB;
  constexpr int NWAVE = NT / 64;
  // wave grid: WC (channel) x WP (pixel) waves; a wave owns WCH channels
  // (64, or all 16 for the narrow NCHW image-grad tile)
  constexpr int WC = BC >= 64 ? BC / 64 : 1, WP = NWAVE / WC, WCH = BC / WC;
  constexpr int MC = WCH / 16, MP = BP / WP / 16;
  constexpr int WPLANE = BC * 16;                               // weight planes: BC rows
  constexpr int WBYTES = 8 * WPLANE;
  constexpr int WPIECES = BC * 8;
  constexpr int LW = (WPIECES + NT - 1) / NT;                   // weight pieces per thread
  constexpr int MAIN = HB * G::HBYTES + 2 * WBYTES;
  constexpr int SROW = BC + 4;
  constexpr int STG = BP * SROW * 4 + 2 * NT * 4 * 2 + 256;
  // the persistent image-grad tile (BC < 64, below): halo + all 9 taps' weights
  constexpr int ONE_BYTES = BC < 64 ? G::HBYTES + 9 * WBYTES : 0;
  static_assert(BC >= 64 || STG <= G::HBYTES, "image-grad staging tile aliases the halo only");
  constexpr int SMEM0 = MAIN > STG ? MAIN : STG;
  constexpr int SMEM = SMEM0 > ONE_BYTES ? SMEM0 : ONE_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  char *const hbuf = smem;                                      // [HB][HBYTES]
  char *const wbuf = smem + HB * G::HBYTES;                     // [2][WBYTES]

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wc = wv % WC, wp = wv / WC;
  // XCD-aware tile order (a.xcd): workgroup b runs on XCD b % 8, so XCD x
  // takes the contiguous tile range [x T/8, (x+1) T/8) -- the column blocks
  // of a pixel tile and the neighbouring tiles sharing its halo rows then
  // meet in one L2.  The remainder (T % 8) keeps the linear order.
  int tile = blockIdx.x;
  if (a.xcd) {
    const int per = (int)gridDim.x / 8;
    if ((int)blockIdx.x < per * 8) tile = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
  }
  const int cblk = tile % a.ncblk, pblk = tile / a.ncblk;
  const int c0 = cblk * BC, p0 = pblk * BP;

  // ---- tile geometry (uniform) ----
  const int hw = a.h * a.w;
  const int n0 = p0 / hw;
  const int y0 = (p0 - n0 * hw) / W;
  const int Hs = G::R < a.h ? G::R : a.h;
  const int himg = (Hs + 2) * (W + 2);                          // halo rows per image
  const int hrows = (G::R / Hs) * himg;

  // ---- per-piece halo source pixel (-1: zero padding), fixed for the tile ----
  int hpix[G::LH];
#pragma unroll
  for (int i = 0; i < G::LH; ++i) {
    const int idx = tid + NT * i;
    const int r = 8 * (idx >> 6) + (idx & 7);
    int pix = -1;
    if (r < hrows) {
      const int im = r / himg, rem = r - (r / himg) * himg;
      const int hy = rem / (W + 2), hx = rem - (rem / (W + 2)) * (W + 2);
      const int yy = y0 - 1 + hy, xx = hx - 1;
      if (yy >= 0 && yy < a.h && xx >= 0 && xx < W) pix = ((n0 + im) * a.h + yy) * W + xx;
    }
    hpix[i] = pix;
  }
  const int pj = ((tid >> 3) & 7) * 16;                         // this thread's 16-B chunk
  // ---- weight rows ----
  const char *wrow[LW];
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    const int idx = tid + NT * i;
    const int r = 8 * (idx >> 6) + (idx & 7);
    // rows past c_out (the narrow tile's padding) load row 0 and are zeroed
    wrow[i] = a.wt + ((long long)(c0 + r < a.cout ? c0 + r : 0) * a.K) * 2 + pj;
  }

  // ---- per-lane fragment bases ----
  const int frow = lane & 15, fq = lane >> 4;
  int abase[MC], bbase[MP];
#pragma unroll
  for (int mi = 0; mi < MC; ++mi) abase[mi] = fq * WPLANE + (wc * WCH + mi * 16 + frow) * 16;
#pragma unroll
  for (int ni = 0; ni < MP; ++ni) {
    const int q = wp * (BP / WP) + ni * 16 + frow;              // pixel within the tile
    const int r = q / W, x = q % W;
    const int im = r / Hs, rr = r - (r / Hs) * Hs;
    bbase[ni] = fq * G::PLANE + (im * himg + rr * (W + 2) + x) * 16;   // tap (dy,dx) = (-1,-1)
  }

  const int kch = a.cin / 64;
  const int nst = kch * 9;
  typedef uint4 V;

  // Persistent image-grad tile (BC < 64: conv1_1's dgrad into the NCHW fp32
  // image grad, one 64-channel K chunk, one column block).  The one-shot
  // tile was bound by its halo load (a ~50 KB gather, then 4 MFMAs per wave
  // per tap): here each workgroup walks tiles blockIdx.x + k gridDim.x with
  // the NEXT tile's halo loading into registers while the current one
  // computes and stores; the 9 taps' weights (9 x 2 KB) are staged once.
  if constexpr (BC < 64) {
    const int ntile = a.P / BP;
    if (kch == 1 && a.ncblk == 1 && (int)gridDim.x < ntile) {
      char *const wall = smem + G::HBYTES;
      for (int i = tid; i < 9 * WPIECES; i += NT) {
        const int tp = i / WPIECES, idx = i - tp * WPIECES;
        const int r = 8 * (idx >> 6) + (idx & 7), j = (idx >> 3) & 7;
        const bool ok = r < a.cout;
        V v = *reinterpret_cast<const V *>(a.wt + ((long long)(ok ? r : 0) * a.K +
                                                   (long long)tp * a.cin) * 2 + j * 16);
        if (!ok) v = V{0u, 0u, 0u, 0u};
        *reinterpret_cast<V *>(wall + tp * WBYTES + j * WPLANE + r * 16) = v;
      }
      V hr[G::LH];
      const char *src0 = a.x1 + pj;
      auto load_h = [&](int t) __attribute__((always_inline)) {
        const int q0 = t * BP;
        const int tn0 = q0 / hw;
        const int ty0 = (q0 - tn0 * hw) / W;
#pragma unroll
        for (int i = 0; i < G::LH; ++i) {
          const int idx = tid + NT * i;
          const int r = 8 * (idx >> 6) + (idx & 7);
          int pix = -1;
          if (r < hrows) {
            const int im = r / himg, rem = r - (r / himg) * himg;
            const int hy = rem / (W + 2), hx = rem - (rem / (W + 2)) * (W + 2);
            const int yy = ty0 - 1 + hy, xx = hx - 1;
            if (yy >= 0 && yy < a.h && xx >= 0 && xx < W) pix = ((tn0 + im) * a.h + yy) * W + xx;
          }
          const bool ok = pix >= 0;
          V v = *reinterpret_cast<const V *>(src0 + (long long)(ok ? pix : 0) * a.c1 * 2);
          v.x = ok ? v.x : 0u; v.y = ok ? v.y : 0u; v.z = ok ? v.z : 0u; v.w = ok ? v.w : 0u;
          hr[i] = v;
        }
      };
      float *const stg = reinterpret_cast<float *>(smem);          // aliases the halo
      float *const yo = reinterpret_cast<float *>(a.y1);
      const int ncol = min(BC, a.cout);
      int t = (int)blockIdx.x;
      load_h(t);
      for (; t < ntile; t += (int)gridDim.x) {
#pragma unroll
        for (int i = 0; i < G::LH; ++i) {
          const int idx = tid + NT * i;
          const int r = 8 * (idx >> 6) + (idx & 7);
          if (r < hrows) *reinterpret_cast<V *>(hbuf + ((idx >> 3) & 7) * G::PLANE + r * 16) = hr[i];
        }
        __syncthreads();                                   // halo(t) (and the weights) visible
        const int tn = t + (int)gridDim.x;
        if (tn < ntile) load_h(tn);                        // next tile's halo in flight
        f32x4 acc[MC][MP];
#pragma unroll
        for (int mi = 0; mi < MC; ++mi)
#pragma unroll
          for (int ni = 0; ni < MP; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const char *sA = wall + tp * WBYTES;
          const char *sB = hbuf + ((tp / 3) * (W + 2) + tp % 3) * 16;
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            bf16x8 fa[MC], fb[MP];
#pragma unroll
            for (int mi = 0; mi < MC; ++mi)
              fa[mi] = *reinterpret_cast<const bf16x8 *>(sA + abase[mi] + kk * 4 * WPLANE);
#pragma unroll
            for (int ni = 0; ni < MP; ++ni)
              fb[ni] = *reinterpret_cast<const bf16x8 *>(sB + bbase[ni] + kk * 4 * G::PLANE);
#pragma unroll
            for (int mi = 0; mi < MC; ++mi)
#pragma unroll
              for (int ni = 0; ni < MP; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi], fb[ni], acc[mi][ni], 0, 0, 0);
          }
        }
        __syncthreads();                                   // every wave done reading halo(t)
#pragma unroll
        for (int mi = 0; mi < MC; ++mi)
#pragma unroll
          for (int ni = 0; ni < MP; ++ni) {
            const int r = wp * (BP / WP) + ni * 16 + frow;
            const int col = wc * WCH + mi * 16 + fq * 4;
            *reinterpret_cast<f32x4 *>(stg + r * SROW + col) = acc[mi][ni];
          }
        __syncthreads();
        const int q0 = t * BP;
        for (int i = tid; i < ncol * BP; i += NT) {
          const int cl = i / BP, r = i - (i / BP) * BP;
          const int p = q0 + r;
          const int nn = p / hw, rem = p - nn * hw;
          float v = stg[r * SROW + cl] + (a.bias ? a.bias[cl] : 0.f);
          const long long o = ((long long)nn * a.cout + cl) * hw + rem;
          if (a.accumulate) v += yo[o];
          if (a.act == RR_ACT_RELU) v = fmaxf(v, 0.f);
          yo[o] = v;
        }
        __syncthreads();                                   // staging read before halo(t+1) lands
      }
      return;
    }
  }

  V hreg[G::LH];
  // weights prefetched 2 stages ahead (register set = stage parity; 3
  // ahead at BC = 128 measured no faster, r2i_dbgk.jsonl)
  V wr0[LW], wr1[LW];

  auto load_halo = [&](int ch) __attribute__((always_inline)) {
    const int ci0 = ch * 64;
    const bool first = ci0 < a.c1;
    const char *base = first ? a.x1 : a.x2;
    const long long cs = first ? a.c1 : a.c2;
    const char *src0 = base + (long long)(first ? ci0 : ci0 - a.c1) * 2 + pj;
#pragma unroll
    for (int i = 0; i < G::LH; ++i) {
      // padding pieces load pixel 0 (valid, L2-hot) and are zeroed by a
      // select: no divergent branch, no pointer merge across address spaces
      const bool ok = hpix[i] >= 0;
      V v = *reinterpret_cast<const V *>(src0 + (long long)(ok ? hpix[i] : 0) * cs * 2);
      v.x = ok ? v.x : 0u; v.y = ok ? v.y : 0u; v.z = ok ? v.z : 0u; v.w = ok ? v.w : 0u;
      hreg[i] = v;
    }
  };
  // the next chunk's halo, spread over taps 0-6: piece i is issued at tap
  // 7 i / LH.  Issued all at tap 0 by every workgroup at once it was a
  // chip-wide burst (256 x ~100 KB) that the in-order vmcnt wait for the
  // weights two stages later then sat behind
  auto load_halo_part = [&](int ch, auto tapc) __attribute__((always_inline)) {
    constexpr int TAP = decltype(tapc)::value;
    const int ci0 = ch * 64;
    const bool first = ci0 < a.c1;
    const char *base = first ? a.x1 : a.x2;
    const long long cs = first ? a.c1 : a.c2;
    const char *src0 = base + (long long)(first ? ci0 : ci0 - a.c1) * 2 + pj;
#pragma unroll
    for (int i = 0; i < G::LH; ++i) {
      if ((i * 7) / G::LH != TAP) continue;
      const bool ok = hpix[i] >= 0;
      V v = *reinterpret_cast<const V *>(src0 + (long long)(ok ? hpix[i] : 0) * cs * 2);
      v.x = ok ? v.x : 0u; v.y = ok ? v.y : 0u; v.z = ok ? v.z : 0u; v.w = ok ? v.w : 0u;
      hreg[i] = v;
    }
  };
  auto store_halo = [&](int buf) __attribute__((always_inline)) {
    char *d = hbuf + buf * G::HBYTES;
#pragma unroll
    for (int i = 0; i < G::LH; ++i) {
      const int idx = tid + NT * i;
      const int r = 8 * (idx >> 6) + (idx & 7);
      if (r < hrows) *reinterpret_cast<V *>(d + ((idx >> 3) & 7) * G::PLANE + r * 16) = hreg[i];
    }
  };
  auto load_w = [&](int s, auto setc) __attribute__((always_inline)) {
    const int ch = s / 9, tap = s - (s / 9) * 9;
    const long long off = ((long long)tap * a.cin + ch * 64) * 2;
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      V v = *reinterpret_cast<const V *>(wrow[i] + off);
      if constexpr (BC < 64) {
        const int idx = tid + NT * i;
        const bool ok = c0 + 8 * (idx >> 6) + (idx & 7) < a.cout;
        v.x = ok ? v.x : 0u; v.y = ok ? v.y : 0u; v.z = ok ? v.z : 0u; v.w = ok ? v.w : 0u;
      }
      if constexpr (decltype(setc)::value == 0) wr0[i] = v;
      else wr1[i] = v;
    }
  };
  // LDS weight buffer SET (stage parity) <- register set REG
  auto store_w = [&](auto setc, auto regc) __attribute__((always_inline)) {
    constexpr int SET = decltype(setc)::value;
    constexpr int REG = decltype(regc)::value;
    char *d = wbuf + SET * WBYTES;
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const int idx = tid + NT * i;
      const int r = 8 * (idx >> 6) + (idx & 7);
      if (WPIECES % NT == 0 || idx < WPIECES)
        *reinterpret_cast<V *>(d + ((idx >> 3) & 7) * WPLANE + r * 16) =
            REG == 0 ? wr0[i] : wr1[i];
    }
  };

  f32x4 acc[MC][MP];
#pragma unroll
  for (int mi = 0; mi < MC; ++mi)
#pragma unroll
    for (int ni = 0; ni < MP; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: halo(0), weights(0) into LDS; weights(1) in flight
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // RS (role split, HB = 2): waves 0-3 stage the weights, waves 4-7 the
  // next chunk's halo.  vmcnt retires in issue order, so a wave that loaded
  // the (HBM, long-latency) halo at tap 0 and then waited for its weights
  // two stages later also waited for the halo: the weight prefetch, not the
  // MFMAs, then set the pace (round-2 halo_dbgk measurement: without the halo loads the
  // K loop ran 9-33% faster).  With separate roles no wave ever waits for a
  // load of the other kind; every wave still runs the same MFMAs.
  // weight/halo role split: measured 3 % faster at BC = 64, W = 32 / 16
  // (r2h_dbgk.jsonl) but 5-7 % slower at BC = 128 (the four weight waves
  // then carry 2 x 4 loads + LDS stores per stage and become the critical
  // path); BC = 64 at W = 64 / 8 spills with it (128-VGPR cap)
  constexpr bool RS = NT == 512 && BC == 64 && (W == 16 || W == 32);
  if constexpr (!RS) {
    load_halo(0);
    load_w(0, I0{});
    load_w(nst > 1 ? 1 : 0, I1{});
    store_halo(0);
    store_w(I0{}, I0{});
    __syncthreads();
  }

  // One (chunk, tap) stage s = 9 ch + TAP.  weights(k) live in register set
  // k & 1: stage s loads weights(s + 2) into set s & 1 (freed when weights(s)
  // was stored) and stores weights(s + 1) from set (s + 1) & 1.  Every load
  // is unconditional (indices clamped at the tail) so no register is a
  // branch merge and the compiler can keep the loads in flight.
  auto stage = [&](int ch, auto tapc, auto setc) __attribute__((always_inline)) {
    constexpr int TAP = decltype(tapc)::value;
    constexpr int SET = decltype(setc)::value;        // == s & 1
    const int s = ch * 9 + TAP;
    load_w(s + 2 < nst ? s + 2 : nst - 1, setc);
    if constexpr (HB == 2) {       // (BC = 64 at its VGPR cap: spills)
      if constexpr (TAP < 7) load_halo_part(ch + 1 < kch ? ch + 1 : ch, tapc);
    } else if constexpr (TAP == 0) {
      if constexpr (HB == 2) load_halo(ch + 1 < kch ? ch + 1 : ch);
      else if (kch > 1) load_halo(ch + 1 < kch ? ch + 1 : ch);   // uniform: kch per launch
    }
    const char *sA = wbuf + SET * WBYTES;
    const char *sB = hbuf + (HB == 2 ? (ch & 1) * G::HBYTES : 0) + ((TAP / 3) * (W + 2) + TAP % 3) * 16;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[MC], fb[MP];
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
        fa[mi] = *reinterpret_cast<const bf16x8 *>(sA + abase[mi] + kk * 4 * WPLANE);
#pragma unroll
      for (int ni = 0; ni < MP; ++ni)
        fb[ni] = *reinterpret_cast<const bf16x8 *>(sB + bbase[ni] + kk * 4 * G::PLANE);
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int ni = 0; ni < MP; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi], fb[ni], acc[mi][ni], 0, 0, 0);
    }
    if (s + 1 < nst)
      store_w(std::integral_constant<int, SET ^ 1>{}, std::integral_constant<int, SET ^ 1>{});
    if constexpr (TAP == 8) {
      if (ch + 1 < kch) {
        if constexpr (HB == 1) {
          __syncthreads();   // every wave is done reading this chunk's halo
          store_halo(0);
        } else {
          store_halo((ch + 1) & 1);
        }
      }
    }
    __syncthreads();
  };
  auto chunk_even = [&](int ch) __attribute__((always_inline)) {          // 9 ch even: s & 1 == TAP & 1
    stage(ch, std::integral_constant<int, 0>{}, I0{});
    stage(ch, std::integral_constant<int, 1>{}, I1{});
    stage(ch, std::integral_constant<int, 2>{}, I0{});
    stage(ch, std::integral_constant<int, 3>{}, I1{});
    stage(ch, std::integral_constant<int, 4>{}, I0{});
    stage(ch, std::integral_constant<int, 5>{}, I1{});
    stage(ch, std::integral_constant<int, 6>{}, I0{});
    stage(ch, std::integral_constant<int, 7>{}, I1{});
    stage(ch, std::integral_constant<int, 8>{}, I0{});
  };
  auto chunk_odd = [&](int ch) __attribute__((always_inline)) {           // 9 ch odd: s & 1 == (TAP + 1) & 1
    stage(ch, std::integral_constant<int, 0>{}, I1{});
    stage(ch, std::integral_constant<int, 1>{}, I0{});
    stage(ch, std::integral_constant<int, 2>{}, I1{});
    stage(ch, std::integral_constant<int, 3>{}, I0{});
    stage(ch, std::integral_constant<int, 4>{}, I1{});
    stage(ch, std::integral_constant<int, 5>{}, I0{});
    stage(ch, std::integral_constant<int, 6>{}, I1{});
    stage(ch, std::integral_constant<int, 7>{}, I0{});
    stage(ch, std::integral_constant<int, 8>{}, I1{});
  };
  if constexpr (!RS) {
    int ch = 0;
    for (; ch + 2 <= kch; ch += 2) {
      chunk_even(ch);
      chunk_odd(ch + 1);
    }
    if (ch < kch) chunk_even(ch);
  } else {
    // weight waves: half of them at BC = 128 (2 x 4 pieces vs 13 halo
    // pieces per thread), a quarter at BC = 64 (2 x 4 vs 8: the same
    // registers as the unsplit kernel, which sits at its 128-VGPR cap)
    constexpr int WT = (HB == 2 ? NWAVE / 2 : NWAVE / 4) * 64;   // weight threads
    constexpr int HT = NT - WT;                                   // halo threads
    constexpr int LH2 = (G::HMAX * 8 + HT - 1) / HT;              // halo pieces per halo thread
    constexpr int LW2 = (WPIECES + WT - 1) / WT;                  // weight pieces per weight thread
    constexpr int NU = LH2 > 2 * LW2 ? LH2 : 2 * LW2;
    constexpr int NPI = LH2 > LW2 ? LH2 : LW2;
    const bool wrole = tid < WT;                                  // wave-uniform
    const int lt = wrole ? tid : tid - WT;
    // per-piece source: halo role -> pixel (-1 = zero padding), weight role
    // -> byte offset of the weight row (+ this thread's 16-B chunk)
    int pidx[NPI];
    V lr[NU];
#pragma unroll
    for (int i = 0; i < NPI; ++i) {
      const int idx = lt + (wrole ? WT : HT) * i;
      const int r = 8 * (idx >> 6) + (idx & 7);
      int v = -1;
      if (wrole) {
        v = (int)(((long long)(c0 + r < a.cout ? c0 + r : 0) * a.K) * 2 + pj);
      } else if (r < hrows) {
        const int im = r / himg, rem = r - (r / himg) * himg;
        const int hy = rem / (W + 2), hx = rem - (rem / (W + 2)) * (W + 2);
        const int yy = y0 - 1 + hy, xx = hx - 1;
        if (yy >= 0 && yy < a.h && xx >= 0 && xx < W) v = ((n0 + im) * a.h + yy) * W + xx;
      }
      pidx[i] = v;
    }
    auto rs_load_halo = [&](int ch) __attribute__((always_inline)) {
      const int ci0 = ch * 64;
      const bool first = ci0 < a.c1;
      const char *base = first ? a.x1 : a.x2;
      const long long cs = first ? a.c1 : a.c2;
      const char *src0 = base + (long long)(first ? ci0 : ci0 - a.c1) * 2 + pj;
#pragma unroll
      for (int i = 0; i < LH2; ++i) {
        const bool ok = pidx[i] >= 0;
        V v = *reinterpret_cast<const V *>(src0 + (long long)(ok ? pidx[i] : 0) * cs * 2);
        v.x = ok ? v.x : 0u; v.y = ok ? v.y : 0u; v.z = ok ? v.z : 0u; v.w = ok ? v.w : 0u;
        lr[i] = v;
      }
    };
    auto rs_store_halo = [&](int buf) __attribute__((always_inline)) {
      char *d = hbuf + buf * G::HBYTES;
#pragma unroll
      for (int i = 0; i < LH2; ++i) {
        const int idx = lt + HT * i;
        const int r = 8 * (idx >> 6) + (idx & 7);
        if (r < hrows) *reinterpret_cast<V *>(d + ((idx >> 3) & 7) * G::PLANE + r * 16) = lr[i];
      }
    };
    auto rs_load_w = [&](int s, auto setc) __attribute__((always_inline)) {
      constexpr int SET = decltype(setc)::value;
      const int ch = s / 9, tap = s - (s / 9) * 9;
      const long long off = ((long long)tap * a.cin + ch * 64) * 2;
#pragma unroll
      for (int i = 0; i < LW2; ++i) lr[SET * LW2 + i] = *reinterpret_cast<const V *>(a.wt + pidx[i] + off);
    };
    auto rs_store_w = [&](auto setc) __attribute__((always_inline)) {
      constexpr int SET = decltype(setc)::value;
      char *d = wbuf + SET * WBYTES;
#pragma unroll
      for (int i = 0; i < LW2; ++i) {
        const int idx = lt + WT * i;
        const int r = 8 * (idx >> 6) + (idx & 7);
        if (WPIECES % WT == 0 || idx < WPIECES)
          *reinterpret_cast<V *>(d + ((idx >> 3) & 7) * WPLANE + r * 16) = lr[SET * LW2 + i];
      }
    };
    // one stage of one role (ROLE 0 weights, 1 halo); SET == s & 1
    auto rs_stage = [&](int ch, auto tapc, auto setc, auto rolec) __attribute__((always_inline)) {
      constexpr int TAP = decltype(tapc)::value;
      constexpr int SET = decltype(setc)::value;
      constexpr int ROLE = decltype(rolec)::value;
      const int s = ch * 9 + TAP;
      if constexpr (ROLE == 0) rs_load_w(s + 2 < nst ? s + 2 : nst - 1, setc);
      if constexpr (ROLE == 1 && TAP == 0) {
        if (HB == 2 || kch > 1) rs_load_halo(ch + 1 < kch ? ch + 1 : ch);   // uniform: kch per launch
      }
      const char *sA = wbuf + SET * WBYTES;
      const char *sB = hbuf + (HB == 2 ? (ch & 1) * G::HBYTES : 0) + ((TAP / 3) * (W + 2) + TAP % 3) * 16;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 fa[MC], fb[MP];
#pragma unroll
        for (int mi = 0; mi < MC; ++mi)
          fa[mi] = *reinterpret_cast<const bf16x8 *>(sA + abase[mi] + kk * 4 * WPLANE);
#pragma unroll
        for (int ni = 0; ni < MP; ++ni)
          fb[ni] = *reinterpret_cast<const bf16x8 *>(sB + bbase[ni] + kk * 4 * G::PLANE);
#pragma unroll
        for (int mi = 0; mi < MC; ++mi)
#pragma unroll
          for (int ni = 0; ni < MP; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi], fb[ni], acc[mi][ni], 0, 0, 0);
      }
      if constexpr (ROLE == 0) {
        if (s + 1 < nst) rs_store_w(std::integral_constant<int, SET ^ 1>{});
      }
      if constexpr (TAP == 8) {
        if (ch + 1 < kch) {
          if constexpr (HB == 1) {
            __syncthreads();                 // every wave is done reading this chunk's halo
            if constexpr (ROLE == 1) rs_store_halo(0);
          } else if constexpr (ROLE == 1) {
            rs_store_halo((ch + 1) & 1);
          }
        }
      }
      __syncthreads();
    };
    auto rs_run = [&](auto rolec) __attribute__((always_inline)) {
      constexpr int ROLE = decltype(rolec)::value;
      using R = std::integral_constant<int, ROLE>;
      auto even = [&](int ch) __attribute__((always_inline)) {
        rs_stage(ch, std::integral_constant<int, 0>{}, I0{}, R{});
        rs_stage(ch, std::integral_constant<int, 1>{}, I1{}, R{});
        rs_stage(ch, std::integral_constant<int, 2>{}, I0{}, R{});
        rs_stage(ch, std::integral_constant<int, 3>{}, I1{}, R{});
        rs_stage(ch, std::integral_constant<int, 4>{}, I0{}, R{});
        rs_stage(ch, std::integral_constant<int, 5>{}, I1{}, R{});
        rs_stage(ch, std::integral_constant<int, 6>{}, I0{}, R{});
        rs_stage(ch, std::integral_constant<int, 7>{}, I1{}, R{});
        rs_stage(ch, std::integral_constant<int, 8>{}, I0{}, R{});
      };
      auto odd = [&](int ch) __attribute__((always_inline)) {
        rs_stage(ch, std::integral_constant<int, 0>{}, I1{}, R{});
        rs_stage(ch, std::integral_constant<int, 1>{}, I0{}, R{});
        rs_stage(ch, std::integral_constant<int, 2>{}, I1{}, R{});
        rs_stage(ch, std::integral_constant<int, 3>{}, I0{}, R{});
        rs_stage(ch, std::integral_constant<int, 4>{}, I1{}, R{});
        rs_stage(ch, std::integral_constant<int, 5>{}, I0{}, R{});
        rs_stage(ch, std::integral_constant<int, 6>{}, I1{}, R{});
        rs_stage(ch, std::integral_constant<int, 7>{}, I0{}, R{});
        rs_stage(ch, std::integral_constant<int, 8>{}, I1{}, R{});
      };
      // prologue: halo(0) (halo role), weights(0) into LDS and weights(1) in
      // flight (weight role)
      if constexpr (ROLE == 1) {
        rs_load_halo(0);
        rs_store_halo(0);
      } else {
        rs_load_w(0, I0{});
        rs_load_w(nst > 1 ? 1 : 0, I1{});
        rs_store_w(I0{});
      }
      __syncthreads();
      int ch = 0;
      for (; ch + 2 <= kch; ch += 2) {
        even(ch);
        odd(ch + 1);
      }
      if (ch < kch) even(ch);
    };
    if (wrole) rs_run(I0{});
    else rs_run(I1{});
  }

  // ---- epilogue: fp32 tile into LDS, then the shared staged store ----
  float *stg = reinterpret_cast<float *>(smem);
#pragma unroll
  for (int mi = 0; mi < MC; ++mi)
#pragma unroll
    for (int ni = 0; ni < MP; ++ni) {
      const int r = wp * (BP / WP) + ni * 16 + frow;
      const int col = wc * WCH + mi * 16 + fq * 4;
      *reinterpret_cast<f32x4 *>(stg + r * SROW + col) = acc[mi][ni];
    }
  __syncthreads();
  if constexpr (BC < 64) {
    // model-boundary image grad: fp32 NCHW, the tile's pixels are whole rows
    // so each channel plane segment is contiguous
    float *yo = reinterpret_cast<float *>(a.y1);
    const int ncol = min(BC, a.cout - c0);
    for (int i = tid; i < ncol * BP; i += NT) {
      const int cl = i / BP, r = i - (i / BP) * BP;
      const int p = p0 + r;
      if (p >= a.P) continue;
      const int nn = p / hw, rem = p - nn * hw;
      float v = stg[r * SROW + cl] + (a.bias ? a.bias[c0 + cl] : 0.f);
      const long long o = ((long long)nn * a.cout + c0 + cl) * hw + rem;
      if (a.accumulate) v += yo[o];
      if (a.act == RR_ACT_RELU) v = fmaxf(v, 0.f);
      yo[o] = v;
    }
  } else {
    store_staged<T, BC, BP, NT, MODE>(a, stg, c0, p0, pblk, tid);
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

// halo path eligibility (bf16 3x3, whole-row 256-pixel tiles); returns BC or 0
int halo_bc(const rr_igemm_desc *d) {
  // RR_PATH igemm_halo=0: the per-tap tiled kernel instead (tests)
  if (!rr_path("igemm_halo", 1) || d->dtype != RR_BF16 || d->mode != RR_CONV3X3) return 0;
  // NCHW fp32 output only through the narrow 16-column tile (image grads)
  if (d->out_nchw && (d->c_out > 16 || d->want_stats || d->c_in2)) return 0;
  const int W = d->w;
  if (!(W == 8 || W == 16 || W == 32 || W == 64)) return 0;
  const int R = 256 / W;
  if (d->h % 8) return 0;
  if (R <= d->h ? (d->h % R) : (R % d->h || d->n % (R / d->h))) return 0;
  if (d->c_in1 % 64 || d->c_in2 % 64) return 0;
  if (d->out_nchw) return 16;
  // BC = 64 (2 WG/CU) up to 128 input channels: the per-tile prologue /
  // epilogue then dominates and overlap wins (measured best, tools/ab_igemm.py)
  const bool wide_ok = d->c_out % 128 == 0 && (d->out_split == 0 || d->out_split % 128 == 0);
  if (wide_ok && d->c_in1 + d->c_in2 > 128) return 128;
  if (d->c_out % 64 == 0) return 64;
  return 0;
}

template <int BC, int BP, int NT = 2 * BP>
int launch_halo(const rr_igemm_desc *d, IgemmArgs &a, hipStream_t st) {
  a.ncblk = (a.cout + BC - 1) / BC;
  const long long nblk = (long long)(a.P / BP) * a.ncblk;
  if (nblk > 0x7fffffffLL) return RR_EUNSUPPORTED;
  dim3 grid((unsigned)nblk), block(NT);
  // the image-grad tile runs persistent (2 workgroups per CU, each walking
  // tiles with the next halo in flight) when it has one K chunk
  if constexpr (BC < 64) {
    if (a.cin == 64 && a.ncblk == 1 && nblk > 512) grid = dim3(512);
  }
  switch (d->w) {
    case 64: hipLaunchKernelGGL((igemm3_halo_kernel<BC, 64, RR_CONV3X3, BP, NT>), grid, block, 0, st, a); break;
    case 32: hipLaunchKernelGGL((igemm3_halo_kernel<BC, 32, RR_CONV3X3, BP, NT>), grid, block, 0, st, a); break;
    case 16: hipLaunchKernelGGL((igemm3_halo_kernel<BC, 16, RR_CONV3X3, BP, NT>), grid, block, 0, st, a); break;
    default: hipLaunchKernelGGL((igemm3_halo_kernel<BC, 8, RR_CONV3X3, BP, NT>), grid, block, 0, st, a); break;
  }
  RR_CHECK_LAUNCH();
  return RR_OK;
}

template <typename T>
int dispatch(const rr_igemm_desc *d, IgemmArgs &a, hipStream_t st) {
  if constexpr (sizeof(T) == 2) {
    const int hb = halo_bc(d);
    if (hb == 128) return launch_halo<128, 256>(d, a, st);
    if (hb == 64) return launch_halo<64, 256>(d, a, st);
    if (hb == 16) return launch_halo<16, 256>(d, a, st);
  }
  const Tile t = pick_tile(d);
  if (t.bc == 128) return launch_mode<T, 128, 128, 2>(d, a, st);
  if (t.bp == 256) return launch_mode<T, 64, 256, 1>(d, a, st);
  return launch_mode<T, 64, 128, 2>(d, a, st);
}

}  // namespace

extern "C" int rr_igemm_stat_blocks(const rr_igemm_desc *d) {
  if (!d) return RR_EINVAL;
  if (const int sb = stream3_blocks(d, 0)) return sb;
  S1Plan pl;
  if (const int g = stream1_plan(d, &pl)) return g;
  if (const int r = conv3r_stat_blocks(d)) return r;
  const long long P = (long long)d->n * d->h * d->w;
  const int hb = halo_bc(d);
  const int bp = hb ? 256 : pick_tile(d).bp;
  return (int)((P + bp - 1) / bp);
}

static int fill_args(const rr_igemm_desc *d, const void *x1, const void *x2, const void *w,
                     const float *bias, void *y1, void *y2, const void *mask,
                     float *stats_partial, IgemmArgs &a) {
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
  a.xcd = 1;                                   // XCD-aware tile order
  a.ncblk = 1;
  a.bt = nullptr; a.bmean = a.binv = a.baff_s = a.baff_b = a.balpha = nullptr;
  a.bpart = a.bapart = nullptr;
  a.alpha = nullptr;
  a.res = nullptr;
  a.ypool = nullptr;
  a.pidx = nullptr;
  a.ntile = 0;
  return RR_OK;
}

// the kernel rr_igemm would launch for *d (same decisions as rr_igemm /
// dispatch; bench.py names its roofline kernel and the tests assert the
// benched schedule with it).  Static strings, never NULL.
extern "C" const char *rr_igemm_kernel_name(const rr_igemm_desc *d, int bnbwd) {
  if (!d) return "invalid";
  if (d->act > RR_ACT_RELU) {
    // (the pool epilogue needs a 2x2 window: rr_igemm_ex refuses such maps)
    if ((d->act & RR_ACT_POOL) && (d->h < 2 || d->w < 2)) return "unsupported";
    if (!bnbwd && stream3_ex_ok(d)) return stream3_name(d, "");
    return !bnbwd && conv3r_bc(d) ? conv3r_name(d) : "unsupported";
  }
  if (stream3_blocks(d, bnbwd)) return stream3_name(d, "");
  S1Plan pl;
  if (!bnbwd && stream1_plan(d, &pl)) return stream1_name(pl);
  if (conv3r_bc(d)) return conv3r_name(d);
  if (d->dtype == RR_BF16) {
    const int hb = halo_bc(d);
    if (hb) {
      static const char *names[3][4] = {
          {"igemm3_halo_kernel<16,8>", "igemm3_halo_kernel<16,16>", "igemm3_halo_kernel<16,32>", "igemm3_halo_kernel<16,64>"},
          {"igemm3_halo_kernel<64,8>", "igemm3_halo_kernel<64,16>", "igemm3_halo_kernel<64,32>", "igemm3_halo_kernel<64,64>"},
          {"igemm3_halo_kernel<128,8>", "igemm3_halo_kernel<128,16>", "igemm3_halo_kernel<128,32>", "igemm3_halo_kernel<128,64>"}};
      const int wi = d->w == 8 ? 0 : d->w == 16 ? 1 : d->w == 32 ? 2 : 3;
      const int bi = hb == 16 ? 0 : hb == 64 ? 1 : 2;
      return names[bi][wi];
    }
  }
  const Tile t = pick_tile(d);
  const bool b = d->dtype == RR_BF16;
  static const char *tn[2][3][4] = {
      {{"igemm_kernel<f32,128,128,m0>", "igemm_kernel<f32,128,128,m1>", "igemm_kernel<f32,128,128,m2>", "igemm_kernel<f32,128,128,m3>"},
       {"igemm_kernel<f32,64,256,m0>", "igemm_kernel<f32,64,256,m1>", "igemm_kernel<f32,64,256,m2>", "igemm_kernel<f32,64,256,m3>"},
       {"igemm_kernel<f32,64,128,m0>", "igemm_kernel<f32,64,128,m1>", "igemm_kernel<f32,64,128,m2>", "igemm_kernel<f32,64,128,m3>"}},
      {{"igemm_kernel<bf16,128,128,m0>", "igemm_kernel<bf16,128,128,m1>", "igemm_kernel<bf16,128,128,m2>", "igemm_kernel<bf16,128,128,m3>"},
       {"igemm_kernel<bf16,64,256,m0>", "igemm_kernel<bf16,64,256,m1>", "igemm_kernel<bf16,64,256,m2>", "igemm_kernel<bf16,64,256,m3>"},
       {"igemm_kernel<bf16,64,128,m0>", "igemm_kernel<bf16,64,128,m1>", "igemm_kernel<bf16,64,128,m2>", "igemm_kernel<bf16,64,128,m3>"}}};
  const int ti = t.bc == 128 ? 0 : (t.bp == 256 ? 1 : 2);
  const int mi = d->mode >= 0 && d->mode <= 3 ? d->mode : 0;
  return tn[b][ti][mi];
}

extern "C" int rr_igemm(const rr_igemm_desc *d, const void *x1, const void *x2,
                        const void *w, const float *bias, void *y1, void *y2,
                        const void *mask, float *stats_partial, rr_stream stream) {
  if (d && (d->act < 0 || d->act > RR_ACT_RELU)) return RR_EINVAL;   // (PReLU / residual: rr_igemm_ex)
  IgemmArgs a;
  const int rc = fill_args(d, x1, x2, w, bias, y1, y2, mask, stats_partial, a);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (stream3_blocks(d, 0)) {
    S3Args s{};
    s.x = a.x1; s.x2 = a.x2; s.wt = a.wt; s.bias = a.bias; s.y = a.y1;
    s.mask = d->has_mask ? a.mask : nullptr;
    s.stats = a.stats;
    s.n = d->n; s.h = d->h; s.w = d->w; s.act = d->act; s.accumulate = d->accumulate;
    return stream3_launch(d, s, 0, st);
  }
  S1Plan pl;
  if (stream1_plan(d, &pl)) {
    S1Args s{};
    s.x1 = a.x1; s.x2 = a.x2; s.wt = a.wt; s.bias = a.bias; s.y1 = a.y1; s.y2 = a.y2;
    s.mask = d->has_mask ? a.mask : nullptr;
    s.stats = a.stats;
    return stream1_launch(d, pl, s, st);
  }
  if (conv3r_bc(d)) return conv3r_launch(d, a, st);
  if (d->dtype == RR_BF16) return dispatch<bf16_t>(d, a, st);
  return dispatch<float>(d, a, st);
}

extern "C" int rr_igemm_ex(const rr_igemm_desc *d, const void *x1, const void *x2, const void *w,
                           const float *bias, const float *alpha, const void *res, void *y1,
                           void *y_pool, const void *mask, float *stats_partial, rr_stream stream) {
  const int all = RR_ACT_RELU | RR_ACT_PRELU | RR_ACT_RES | RR_ACT_POOL | RR_ACT_NOFULL;
  if (!d || d->act < 0 || (d->act & ~all) || (d->act & 3) == 3) return RR_EINVAL;
  if ((d->act & 3) == RR_ACT_PRELU && !alpha) return RR_EINVAL;
  if ((d->act & RR_ACT_RES) && (!res || d->out_split || d->accumulate || d->out_nchw)) return RR_EINVAL;
  if ((d->act & RR_ACT_POOL) && (!y_pool || d->out_split || d->h < 2 || d->w < 2)) return RR_EINVAL;
  if ((d->act & RR_ACT_NOFULL) && (!(d->act & RR_ACT_POOL) || d->accumulate || d->want_stats))
    return RR_EINVAL;
  if (d->act > RR_ACT_RELU && stream3_ex_ok(d)) {
    // the 64 -> 64 maps the streaming kernel takes (whole rows, or column
    // strips of the reference's 224 maps)
    if (!x1 || !w || !bias || (!y1 && !(d->act & RR_ACT_NOFULL))) return RR_EINVAL;
    S3Args s{};
    s.x = (const char *)x1; s.wt = (const char *)w; s.bias = bias;
    s.y = (d->act & RR_ACT_NOFULL) ? nullptr : (char *)y1;
    s.n = d->n; s.h = d->h; s.w = d->w; s.act = d->act;
    s.alpha = alpha; s.res = (const char *)res; s.ypool = (char *)y_pool;
    return stream3_launch_ex(d, s, (hipStream_t)stream);
  }
  if (d->act > RR_ACT_RELU && !conv3r_bc(d)) return RR_EUNSUPPORTED;
  // (y1 unused with RR_ACT_NOFULL: fill_args wants a pointer)
  void *y1a = (d->act & RR_ACT_NOFULL) ? y_pool : y1;
  IgemmArgs a;
  const int rc = fill_args(d, x1, x2, w, bias, y1a, nullptr, mask, stats_partial, a);
  if (rc) return rc;
  if (d->act <= RR_ACT_RELU) {
    rr_igemm_desc d2 = *d;
    return rr_igemm(&d2, x1, x2, w, bias, y1, nullptr, mask, stats_partial, stream);
  }
  a.alpha = alpha;
  a.res = (const char *)res;
  a.ypool = (char *)y_pool;
  return conv3r_launch(d, a, (hipStream_t)stream);
}

// conv2's bias + BN-statistics forward with BN1 + PReLU of its input folded
// in (x1 = t1; the conv reads PReLU(t1 * pre_scale + pre_shift), the bytes
// rr_affine_act would store): the row-streaming kernel's 64 -> 64 whole-row
// maps only (rr_igemm_pre_ok)
extern "C" int rr_igemm_pre_ok(const rr_igemm_desc *d) {
  return d && d->mode == RR_CONV3X3 && d->act == RR_ACT_NONE && d->has_bias && d->want_stats &&
                 !d->accumulate && !d->has_mask && !d->c_in2 && stream3_blocks(d, 0) && !stream3_strips(d)
             ? 1
             : 0;
}

extern "C" int rr_igemm_pre(const rr_igemm_desc *d, const void *x1, const void *w, const float *bias,
                            const float *pre_scale, const float *pre_shift, const float *pre_alpha,
                            void *y1, float *stats_partial, rr_stream stream) {
  if (!d || !x1 || !w || !bias || !pre_scale || !pre_shift || !pre_alpha || !y1 || !stats_partial)
    return RR_EINVAL;
  if (!rr_igemm_pre_ok(d)) return RR_EUNSUPPORTED;
  S3Args s{};
  s.x = (const char *)x1; s.wt = (const char *)w; s.bias = bias; s.y = (char *)y1;
  s.stats = stats_partial;
  s.n = d->n; s.h = d->h; s.w = d->w; s.act = d->act;
  s.pre_s = pre_scale; s.pre_b = pre_shift; s.pre_alpha = pre_alpha;
  return stream3_launch_pre(d, s, (hipStream_t)stream);
}

// conv (+ bias) + ReLU + MaxPool2d(2, 2) with the window index, the full-size
// output never written (the perceptual VGG slice's conv1_2 / conv2_2 + pool,
// 14:189-196, and every no-backward pool of it): the row-streaming kernel
// where it takes the layer, else the tap-reuse conv's register epilogue
extern "C" int rr_igemm_pool(const rr_igemm_desc *d, const void *x1, const void *x2, const void *w,
                             const float *bias, void *y_pool, uint8_t *pool_idx, rr_stream stream) {
  if (!d || !y_pool || d->mode != RR_CONV3X3 || d->act != RR_ACT_RELU || d->out_split ||
      d->accumulate || d->has_mask || d->want_stats || d->out_nchw || d->h < 2 || d->w < 2)
    return RR_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (stream3_blocks(d, 0) && !d->c_in2 && (pool_idx ? !stream3_strips(d) : d->has_bias)) {
    S3Args s{};
    s.x = (const char *)x1; s.wt = (const char *)w; s.bias = d->has_bias ? bias : nullptr;
    s.n = d->n; s.h = d->h; s.w = d->w; s.act = d->act;
    s.ypool = (char *)y_pool; s.pidx = pool_idx;
    if (!x1 || !w || (d->has_bias && !bias)) return RR_EINVAL;
    return stream3_launch_pool(d, s, st);
  }
  rr_igemm_desc d2 = *d;
  d2.act = RR_ACT_RELU | RR_ACT_POOL | RR_ACT_NOFULL;
  if (!conv3r_bc(&d2)) return RR_EUNSUPPORTED;
  IgemmArgs a;
  const int rc = fill_args(&d2, x1, x2, w, bias, y_pool, nullptr, nullptr, nullptr, a);
  if (rc) return rc;
  a.ypool = (char *)y_pool;
  a.pidx = pool_idx;
  return conv3r_launch(&d2, a, st);
}

// the kernel rr_igemm_pool launches for *d ("unsupported" when neither takes it)
extern "C" const char *rr_igemm_pool_kernel_name(const rr_igemm_desc *d) {
  if (!d || d->mode != RR_CONV3X3 || d->act != RR_ACT_RELU || d->out_split || d->accumulate ||
      d->has_mask || d->want_stats || d->out_nchw || d->h < 2 || d->w < 2)
    return "unsupported";
  if (stream3_blocks(d, 0) && !d->c_in2) return stream3_name(d, "pool");
  rr_igemm_desc d2 = *d;
  d2.act = RR_ACT_RELU | RR_ACT_POOL | RR_ACT_NOFULL;
  return conv3r_bc(&d2) ? conv3r_name(&d2) : "unsupported";
}

// the 3x3 dgrad plus the 1x1 dgrad of a second gradient into one output, one
// pass: a ResidualBlock's input grad is conv_block[0]'s dgrad + shortcut[0]'s
// dgrad (14:99-115) -- dec1 (64 + 64 -> 64): per concat half, instead of a
// 3x3 dgrad and a 1x1 accumulate pass over both halves
static bool dgrad_sc_ok(const rr_igemm_desc *d, int c_sc) {
  return d && d->mode == RR_CONV3X3 && !d->act && !d->has_bias && !d->want_stats && !d->has_mask &&
         !d->out_split && !d->accumulate && !d->out_nchw && !d->c_in2 && c_sc == 64 &&
         stream3_blocks(d, 0) && !stream3_strips(d);
}

extern "C" int rr_igemm_dgrad_sc(const rr_igemm_desc *d, const void *dy, const void *w,
                                 const void *dy_sc, const void *w_sc, int c_sc, void *y,
                                 rr_stream stream) {
  if (!d || !dy || !w || !dy_sc || !w_sc || !y || c_sc <= 0) return RR_EINVAL;
  if (d->mode != RR_CONV3X3 || d->act || d->has_bias || d->want_stats || d->has_mask ||
      d->out_split || d->accumulate || d->out_nchw || d->c_in2)
    return RR_EINVAL;
  if (!dgrad_sc_ok(d, c_sc)) return RR_EUNSUPPORTED;
  S3Args s{};
  s.x = (const char *)dy; s.wt = (const char *)w; s.y = (char *)y;
  s.n = d->n; s.h = d->h; s.w = d->w;
  s.xsc = (const char *)dy_sc; s.wsc = (const char *)w_sc;
  return stream3_launch_sc(d, s, (hipStream_t)stream);
}

extern "C" const char *rr_igemm_dgrad_sc_kernel_name(const rr_igemm_desc *d, int c_sc) {
  if (!dgrad_sc_ok(d, c_sc)) return "unsupported";
  return stream3_name(d, "sc");
}

static int bnbwd_rows(const rr_igemm_desc *d) { return rr_igemm_stat_blocks(d); }

extern "C" size_t rr_igemm_bnbwd_workspace(const rr_igemm_desc *d) {
  if (!d || d->c_out <= 0) return 0;
  const int rows = bnbwd_rows(d);
  if (rows <= 0) return 0;
  return ((size_t)rows * d->c_out * 3 + (size_t)rows * (d->c_out / 64)) * sizeof(float);
}

extern "C" int rr_igemm_bnbwd(const rr_igemm_desc *d, const void *dy, const void *w,
                              const void *t, const float *mean, const float *invstd,
                              const float *aff_s, const float *aff_b, const float *alpha,
                              void *gm_out, float *partial, rr_stream stream) {
  if (!d || !dy || !w || !t || !mean || !invstd || !aff_s || !aff_b || !alpha || !gm_out ||
      !partial)
    return RR_EINVAL;
  if (d->mode != RR_CONV3X3 && d->mode != RR_CONV1X1) return RR_EUNSUPPORTED;
  if (d->c_in2 || d->out_split || d->has_mask || d->accumulate || d->has_bias || d->want_stats ||
      d->out_nchw || d->act)
    return RR_EINVAL;
  if (d->c_out % 64) return RR_EUNSUPPORTED;      // staged epilogue: whole column tiles
  IgemmArgs a;
  const int rc = fill_args(d, dy, nullptr, w, nullptr, gm_out, nullptr, nullptr, nullptr, a);
  if (rc) return rc;
  a.bt = (const char *)t;
  a.bmean = mean; a.binv = invstd; a.baff_s = aff_s; a.baff_b = aff_b; a.balpha = alpha;
  a.bpart = partial;
  a.bapart = partial + (size_t)bnbwd_rows(d) * d->c_out * 3;
  hipStream_t st = (hipStream_t)stream;
  if (stream3_blocks(d, 1)) {
    S3Args s{};
    s.x = a.x1; s.wt = a.wt; s.y = a.y1;
    s.n = d->n; s.h = d->h;
    s.bt = a.bt; s.bmean = mean; s.binv = invstd; s.baff_s = aff_s; s.baff_b = aff_b;
    s.balpha = alpha; s.bpart = a.bpart; s.bapart = a.bapart;
    return stream3_launch(d, s, 1, st);
  }
  if (conv3r_bc(d)) return conv3r_launch(d, a, st);
  if (d->dtype == RR_BF16) return dispatch<bf16_t>(d, a, st);
  return dispatch<float>(d, a, st);
}
