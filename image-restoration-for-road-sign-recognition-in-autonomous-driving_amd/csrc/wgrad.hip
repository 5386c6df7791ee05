// wgrad.hip -- weight-gradient GEMMs on CDNA4 MFMA (gfx950).
//
// Replaces the weight half of ATen convolution_backward for the reference's
// nn.Conv2d (07:78-96, 14:100-111, VGG16 features) and nn.ConvTranspose2d
// (07:88,92, 14:143-149):
//   conv   : dW[co][ci][t] = sum_p dy[p][co] * x[src(p,t)][ci]
//   convT  : dW[ci][co][t] = sum_p x[p][ci]  * dy[up(p,t)][co]
// Both are   D[a][b] (per tap t) = sum_p A[p][a] * B[map_t(p)][b]
// with A read at the GEMM pixel p and B gathered (3x3 halo shift with zero
// padding, identity, or the 2x2 up-scatter position of a transposed conv).
//
// The reduction runs over pixels (K = N*H*W, up to 2M at batch 512 @64^2), so
// it is split over workgroups (split-K): each split writes an fp32 partial
// slab, and a second kernel sums the slabs in a fixed order (bitwise
// reproducible) straight into the torch-layout fp32 gradient.
//
// Tiles: BA x BB outputs per 256-thread workgroup (4 waves, 2x2), 64 pixels
// of K per stage, register-staged global->LDS (16-B loads, 16-B ds_writes)
// into XOR-swizzled [pixel][channel] images, double buffered.  The MFMA
// operands need the K (pixel) index inside a lane's fragment, i.e. a
// transposed read of the pixel-major image:
//   bf16: two ds_read_b64_tr_b16 per fragment (4 pixels each), 16x16x32 MFMA
//   f32 : ds_read_b32 per fragment, 16x16x4 f32 MFMA (exact fp32)
#include "common.h"

#include <type_traits>
#include "swgrad.h"

#include <cstdlib>

namespace {

struct WgradArgs {
  const char *A;           // [P][CA]
  const char *B1, *B2;     // [Pb][c1], [Pb][c2]  (B grid)
  float *partial;          // [nsplit][CA][taps][CB]
  int CA, CB, c1, c2;
  int taps;
  int n, h, w;             // A grid (GEMM pixels)
  int P;
  int split_len;           // pixels per split (multiple of BKP)
  int nablk, nbblk;
  FastDiv fd_w, fd_hw;
  int xcd;                 // XCD-aware workgroup order (always on)
};

// XCD-aware order (workgroup b runs on XCD b % 8): XCD x takes the
// contiguous index range [x T/8, (x+1) T/8), so the tiles of one split --
// which read the same dy / x pixels -- share an L2; the T % 8 tail is linear
__device__ __forceinline__ int xcd_order(int b, int xcd) {
  if (!xcd) return b;
  const int per = (int)gridDim.x / 8;
  return b < per * 8 ? (b & 7) * per + (b >> 3) : b;
}

constexpr int BKP_PLAN = 64;   // split lengths are multiples of this

// byte offset of 16-B piece `piece` of row r in a swizzled [row][RB bytes] image
template <typename T, int RB>
__device__ __forceinline__ int wg_off(int r, int piece) {
  if constexpr (sizeof(T) == 2) {
    // 32-B units (16 bf16 columns = one tr-read block)
    const int u = piece >> 1, h = piece & 1;
    int f;
    if constexpr (RB >= 256) f = (r & 3) | (((r >> 3) & 1) << 2);
    else f = ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
    return r * RB + ((u ^ f) << 5) + (h << 4);
  } else {
    // 64-B units (16 fp32 columns), rows alternate halves of a 128-B bank row
    const int u = piece >> 2, h = piece & 3;
    return r * RB + ((u ^ (r & 1)) << 6) + (h << 4);
  }
}

typedef short s16x8 __attribute__((ext_vector_type(8)));

// bf16 MFMA operand with the K index (pixel) inside the lane: two transposed
// 4x16 block reads (rows k..k+3 and k+4..k+7), concatenated.
__device__ __forceinline__ bf16x8 tr_frag(const char *p0, const char *p1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4 *)LDS_PTR(p0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4 *)LDS_PTR(p1));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

template <typename T, int BA, int BB, int MODE>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgradArgs a) {
  constexpr int ES = sizeof(T);
  constexpr int BKP = 128 / ES;                        // pixels per stage (bf16 64, f32 32)
  constexpr int RBA = BA * ES, RBB = BB * ES;          // row bytes
  constexpr int A_BYTES = BKP * RBA, B_BYTES = BKP * RBB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int PA = RBA / 16, PB = RBB / 16;         // 16-B pieces per row
  constexpr int LA = BKP * PA / 256, LB = BKP * PB / 256;  // loads per thread
  constexpr int MA = BA / 32, MB = BB / 32;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wa = wv & 1, wb = wv >> 1;
  int bid = xcd_order(blockIdx.x, a.xcd);
  const int ablk = bid % a.nablk; bid /= a.nablk;
  const int bt = bid % (a.nbblk * a.taps); bid /= (a.nbblk * a.taps);
  const int split = bid;
  const int tap = bt / a.nbblk;
  const int bblk = bt - tap * a.nbblk;
  const int a0 = ablk * BA, b0 = bblk * BB;
  const int pbeg = split * a.split_len;
  const int pend = min(a.P, pbeg + a.split_len);

  // B source for this tile column range
  const char *Bsrc;
  int ldb, bc0;
  if (b0 < a.c1) { Bsrc = a.B1; ldb = a.c1; bc0 = b0; }
  else { Bsrc = a.B2; ldb = a.c2; bc0 = b0 - a.c1; }
  const int bvalid = min(BB, a.CB - b0);   // valid columns in this tile

  int dyt = 0, dxt = 0;
  if (MODE == RR_CONV3X3) { dyt = tap / 3 - 1; dxt = tap % 3 - 1; }

  typedef uint4 V;
  V ra[LA], rb[LB];

  auto gload = [&](int pk) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + 256 * i;
      const int r = idx / PA, pc = idx % PA;
      const int p = pk + r;
      V v = {0, 0, 0, 0};
      if (p < pend && a0 + pc * (16 / ES) < a.CA)
        v = *reinterpret_cast<const V *>(a.A + ((long long)p * a.CA + a0) * ES + pc * 16);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + 256 * i;
      const int r = idx / PB, pc = idx % PB;
      const int p = pk + r;
      V v = {0, 0, 0, 0};
      if (p < pend && pc * (16 / ES) < bvalid) {
        long long sp;
        bool ok = true;
        if (MODE == RR_CONV3X3) {
          const uint32_t nh = fdiv((uint32_t)p, a.fd_w);      // n*h + hh
          const int ww = p - (int)nh * a.w;
          const uint32_t nn = fdiv((uint32_t)p, a.fd_hw);
          const int hh = (int)nh - (int)nn * a.h;
          const int h2 = hh + dyt, w2 = ww + dxt;
          ok = (h2 >= 0 && h2 < a.h && w2 >= 0 && w2 < a.w);
          sp = (long long)p + dyt * a.w + dxt;
        } else if (MODE == RR_CONV1X1) {
          sp = p;
        } else {  // RR_CONVT_UP: B grid is (2h, 2w)
          const uint32_t nh = fdiv((uint32_t)p, a.fd_w);
          const int ww = p - (int)nh * a.w;
          const uint32_t nn = fdiv((uint32_t)p, a.fd_hw);
          const int hh = (int)nh - (int)nn * a.h;
          sp = ((long long)nn * 2 * a.h + 2 * hh + (tap >> 1)) * (2 * a.w) + 2 * ww + (tap & 1);
        }
        if (ok) v = *reinterpret_cast<const V *>(Bsrc + (sp * ldb + bc0) * ES + pc * 16);
      }
      rb[i] = v;
    }
  };
  auto swrite = [&](int buf) {
    char *sA = smem + buf * STAGE;
    char *sB = sA + A_BYTES;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + 256 * i;
      *reinterpret_cast<V *>(sA + wg_off<T, RBA>(idx / PA, idx % PA)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + 256 * i;
      *reinterpret_cast<V *>(sB + wg_off<T, RBB>(idx / PB, idx % PB)) = rb[i];
    }
  };

  f32x4 acc[MA][MB];
#pragma unroll
  for (int i = 0; i < MA; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nst = (pend - pbeg + BKP - 1) / BKP;
  if (nst > 0) {
    gload(pbeg);
    swrite(0);
    __syncthreads();
  }
  const int g = lane >> 4, gi = lane & 15;
  const int q = gi >> 2, pp = gi & 3;
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    if (s + 1 < nst) gload(pbeg + (s + 1) * BKP);
    const char *sA = smem + buf * STAGE;
    const char *sB = sA + A_BYTES;
    if constexpr (ES == 2) {
#pragma unroll
      for (int kk = 0; kk < BKP / 32; ++kk) {
        bf16x8 fa[MA], fb[MB];
        // pixel rows of this lane's tr-read addresses (k = 8g + 4*half + q)
        const int r0 = kk * 32 + 8 * g + q, r1 = r0 + 4;
#pragma unroll
        for (int i = 0; i < MA; ++i) {
          const int col = wa * (BA / 2) + i * 16;         // 16-column block
          fa[i] = tr_frag(sA + wg_off<T, RBA>(r0, col / 8) + pp * 8,
                          sA + wg_off<T, RBA>(r1, col / 8) + pp * 8);
        }
#pragma unroll
        for (int j = 0; j < MB; ++j) {
          const int col = wb * (BB / 2) + j * 16;
          fb[j] = tr_frag(sB + wg_off<T, RBB>(r0, col / 8) + pp * 8,
                          sB + wg_off<T, RBB>(r1, col / 8) + pp * 8);
        }
#pragma unroll
        for (int i = 0; i < MA; ++i)
#pragma unroll
          for (int j = 0; j < MB; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll 4
      for (int kk = 0; kk < BKP / 4; ++kk) {
        const int r = kk * 4 + g;
        float fa[MA], fb[MB];
#pragma unroll
        for (int i = 0; i < MA; ++i) {
          const int col = wa * (BA / 2) + i * 16 + gi;
          fa[i] = *reinterpret_cast<const float *>(sA + wg_off<T, RBA>(r, col / 4) + (col & 3) * 4);
        }
#pragma unroll
        for (int j = 0; j < MB; ++j) {
          const int col = wb * (BB / 2) + j * 16 + gi;
          fb[j] = *reinterpret_cast<const float *>(sB + wg_off<T, RBB>(r, col / 4) + (col & 3) * 4);
        }
#pragma unroll
        for (int i = 0; i < MA; ++i)
#pragma unroll
          for (int j = 0; j < MB; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
    // buf^1 was last read in stage s-1, which every wave finished before the
    // barrier that closed it: refill it now, one barrier per stage.
    if (s + 1 < nst) swrite(buf ^ 1);
    __syncthreads();
  }

  // partial[split][a / 4][tap][b][a % 4] where a.CA % 4 == 0: the
  // accumulator's own layout, one 16-B store per lane and block (as
  // wgrad3_halo_kernel; rr_wgrad_reduce maps it back), else [split][a][tap][b]
  if (a.CA % 4 == 0) {
#pragma unroll
    for (int i = 0; i < MA; ++i)
#pragma unroll
      for (int j = 0; j < MB; ++j) {
        const int b = b0 + wb * (BB / 2) + j * 16 + gi;
        const int a4 = (a0 + wa * (BA / 2) + i * 16) / 4 + g;
        if (b >= a.CB || b - b0 >= bvalid || a4 * 4 >= a.CA) continue;
        *reinterpret_cast<f32x4 *>(a.partial + ((((long long)split * (a.CA / 4) + a4) * a.taps + tap) * a.CB + b) * 4) =
            acc[i][j];
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < MA; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      const int b = b0 + wb * (BB / 2) + j * 16 + gi;
      if (b >= a.CB || b - b0 >= bvalid) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ar = a0 + wa * (BA / 2) + i * 16 + g * 4 + e;
        if (ar < a.CA)
          a.partial[(((long long)split * a.CA + ar) * a.taps + tap) * a.CB + b] = acc[i][j][e];
      }
    }
}

// ---------------------------------------------------------------------------
// 3x3 bf16 weight grad with an LDS halo: one workgroup owns a 64 x 64
// (a = dy channel, b = x channel) tile for ALL 9 taps.  A K stage is 64
// pixels = R = 64/W whole image rows of one image; it stages dy[64 px][64 ch]
// and the zero-padded x halo [(R+2) rows][(W+2) cols][64 ch] once, and every
// tap reads its B fragments at a shifted halo row (padding = the conv's zero
// padding, so no masking).  Per stage per wave: 36 MFMAs (2 x 2 x 9) for
// 4 + 36 ds_read_b64_tr_b16; global traffic ~4x lower than per-tap tiles.
struct Halo3Args {
  const char *A;           // dy [P][CA]
  const char *B1, *B2;     // x sources [P][c1], [P][c2]
  float *partial;          // [nsplit][CA][9][CB]
  int CA, CB, c1, c2;
  int n, h, w, lw;         // lw = log2(w)
  int stages;              // total 64-pixel stages (P / 64)
  int split_stages;        // stages per split
  int nablk, nbblk;
  int xcd;                 // XCD-aware workgroup order (always on)
};

// MA = 4: each wave owns all 64 dy channels of the tile and 16 x channels, so
// per 32-pixel step it reads 4 A fragments (reused over the 9 taps) and 9 B
// fragments -- 13 transposed fragment reads per 36 MFMAs.
//
// Operands arrive by LDS-DMA (global_load_lds_dwordx4, round 6): a stage is
// the dy tile [64 px][64 ch] and the x halo [(R+2) rows][(W+2) cols][64 ch] as
// 1-KB pieces of 8 LDS rows, the padding pixels from the zero page, three
// stage buffers (two at W = 64), every wave issuing the same number of pieces
// per stage (counted vmcnt waits + a raw barrier).  Until round 6 the stage
// went global -> registers -> ds_write: two register sets of staging (48
// VGPRs), per-element bounds branches, and rows padded to 136 B that left
// every transposed read 2-way bank-conflicted (41 % of the LDS cycles,
// profiles/r6w_pmc_stalls.json).  The rows are now 128 B with the 32-B column
// blocks XOR-swizzled so the 8 rows one ds_read_b64_tr_b16 half-wave touches
// land on disjoint 8-bank windows: dy rows by pixel bits 1 and 3 (the tiled
// kernel's wg_off), halo rows by their column (W >= 16: the half-wave reads
// columns {x..x+3, x+8..x+11} of one row) or by column bit 1 and row parity
// (W = 8: columns {x..x+3} of two consecutive rows).  The DMA writes a row's
// 16-B slots in lane order, so a lane fetches the chunk its slot holds.
template <int N> using ic = std::integral_constant<int, N>;

template <int OFF> __device__ __forceinline__ s16x4 tr_read(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

template <int W>
__global__ __launch_bounds__(256, 2) void wgrad3_halo_kernel(Halo3Args a) {
  constexpr int MA = 4;
  constexpr int R = 64 / W;                    // image rows per stage
  constexpr int HW2 = W + 2;
  constexpr int HROWS = (R + 2) * HW2;         // halo pixel rows
  constexpr int RS = 128;                      // 64 bf16 channels per LDS row
  constexpr int NB = (HROWS + 7) / 8;          // 1-KB halo pieces (8 rows each)
  constexpr int NJ = 8 + NB;                   // pieces per stage (dy: 8)
  constexpr int NI = (NJ + 3) / 4;             // DMA instructions per wave per stage
  constexpr int A_BYTES = 64 * RS;
  constexpr int STAGE = A_BYTES + NB * 8 * RS;
  constexpr int NSTG = 3 * STAGE <= 80 * 1024 ? 3 : 2;   // two workgroups per CU
  static_assert(NI <= 16, "piece classes");
  __shared__ __attribute__((aligned(16))) char smem[NSTG * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wb = wv;                           // the wave's 16 x channels (all 64 dy channels)
  int bid = xcd_order(blockIdx.x, a.xcd);
  const int ablk = bid % a.nablk; bid /= a.nablk;
  const int bblk = bid % a.nbblk; bid /= a.nbblk;
  const int split = bid;
  const int a0 = ablk * 64, b0 = bblk * 64;
  const int sbeg = split * a.split_stages;
  const int send = min(a.stages, sbeg + a.split_stages);
  const char *Bsrc;
  int ldb, bc0;
  if (b0 < a.c1) { Bsrc = a.B1; ldb = a.c1; bc0 = b0; }
  else { Bsrc = a.B2; ldb = a.c2; bc0 = b0 - a.c1; }
  const int hw = a.h * W;

  auto swz_a = [](int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); };
  auto swz_b = [](int hy, int hx) {
    return W == 8 ? (((hx >> 1) & 1) | ((hy & 1) << 1)) : (((hx >> 1) & 1) | (((hx >> 3) & 1) << 1));
  };

  // ---- the lane's DMA pieces: piece j = wv + 4 i (past the last one: a
  // duplicate of the previous wave's, the same bytes written twice) ----
  int doff[NI];                                // source offset from the stage's dy / halo base
  uint64_t dcls = 0;                           // 4 bits per piece: 1 dy, 2 halo, 4 top row, 8 bottom row
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    int j = wv + 4 * i;
    if (j >= NJ) j -= 4;
    const int rl = lane >> 3, p = lane & 7;
    uint64_t cls = 0;
    int off = 0;
    if (j < 8) {
      const int r = 8 * j + rl;
      const int c = (((p >> 1) ^ swz_a(r)) << 1) | (p & 1);
      off = (r * a.CA + a0) * 2 + c * 16;
      cls = 1;
    } else {
      const int rr = 8 * (j - 8) + rl;
      if (rr < HROWS) {
        const int hy = rr / HW2, hx = rr - (rr / HW2) * HW2;
        const int c = (((p >> 1) ^ swz_b(hy, hx)) << 1) | (p & 1);
        if (hx >= 1 && hx <= W) {
          off = ((hy - 1) * W + hx - 1) * ldb * 2 + c * 16;
          cls = hy == 0 ? 4u : (hy == R + 1 ? 8u : 2u);
        }
      }
    }
    doff[i] = off;
    dcls |= cls << (4 * i);
  }
  const char *zp = rr_zero_page;
  auto issue = [&](int st, int buf) __attribute__((always_inline)) {
    const int p0 = st * 64;                    // first pixel of the stage (R whole rows of one image)
    const int nn = p0 / hw;
    const int h0 = (p0 - nn * hw) / W;
    const char *abase = a.A + (long long)p0 * a.CA * 2;
    const char *bbase = Bsrc + ((long long)(nn * a.h + h0) * W) * ldb * 2 + bc0 * 2;
    const uint64_t okm = 1u | 2u | (h0 > 0 ? 4u : 0u) | (h0 + R < a.h ? 8u : 0u);   // uniform
    char *dst = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      int j = wv + 4 * i;
      if (j >= NJ) j -= 4;                     // (uniform)
      const char *base = j < 8 ? abase : bbase;
      const bool ok = ((dcls >> (4 * i)) & okm & 15u) != 0;
      const char *src = ok ? base + doff[i] : zp;
      const int d = j < 8 ? j * 1024 : A_BYTES + (j - 8) * 1024;
      __builtin_amdgcn_global_load_lds((const void *)src, LDS_PTR(dst + d), 16, 0, 0);
    }
  };

  f32x4 acc[MA][9];
#pragma unroll
  for (int i = 0; i < MA; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- tr-read addresses: bases + compile-time offsets (the swizzle of a dy
  // row does not change with kk, 32 pixels; of a halo row it depends on the
  // tap's dx and, at W = 8, flips bit 1 with an odd dy: address bit 6) ----
  const int g = lane >> 4, gi = lane & 15;
  const int q = gi >> 2, pp = gi & 3;
  const int kl0 = 8 * g + q, kl1 = kl0 + 4;            // the lane's pixel rows at kk = 0
  const uint32_t sbase = (uint32_t)(uintptr_t)smem;
  const uint32_t ab0 = kl0 * RS + (swz_a(kl0) << 5) + pp * 8, ab1 = kl1 * RS + (swz_a(kl1) << 5) + pp * 8;
  uint32_t bb0[3], bb1[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int y0 = kl0 / W, x0 = (kl0 & (W - 1)) + dx, y1 = kl1 / W, x1 = (kl1 & (W - 1)) + dx;
    bb0[dx] = A_BYTES + (y0 * HW2 + x0) * RS + ((wb ^ swz_b(y0, x0)) << 5) + pp * 8;
    bb1[dx] = A_BYTES + (y1 * HW2 + x1) * RS + ((wb ^ swz_b(y1, x1)) << 5) + pp * 8;
  }
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const uint32_t sb = sbase + buf * STAGE;
    // the stage's read bases (kk and dy are immediate offsets)
    uint32_t aa[MA][2], ba[2][3][2];
#pragma unroll
    for (int i = 0; i < MA; ++i) { aa[i][0] = sb + (ab0 ^ (i << 5)); aa[i][1] = sb + (ab1 ^ (i << 5)); }
#pragma unroll
    for (int fl = 0; fl < (W == 8 ? 2 : 1); ++fl)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        ba[fl][dx][0] = sb + (bb0[dx] ^ (fl ? 64u : 0u));
        ba[fl][dx][1] = sb + (bb1[dx] ^ (fl ? 64u : 0u));
      }
    auto kloop = [&](auto KKc) __attribute__((always_inline)) {
      constexpr int kk = decltype(KKc)::value;
      s16x4 fa[MA][2];
      s16x4 fb[2][2];
      constexpr int AOFF = kk * 32 * RS;
      fa[0][0] = tr_read<AOFF>(aa[0][0]); fa[0][1] = tr_read<AOFF>(aa[0][1]);
      fa[1][0] = tr_read<AOFF>(aa[1][0]); fa[1][1] = tr_read<AOFF>(aa[1][1]);
      fa[2][0] = tr_read<AOFF>(aa[2][0]); fa[2][1] = tr_read<AOFF>(aa[2][1]);
      fa[3][0] = tr_read<AOFF>(aa[3][0]); fa[3][1] = tr_read<AOFF>(aa[3][1]);
      auto read_b = [&](auto Tc, s16x4 (&o)[2]) __attribute__((always_inline)) {
        constexpr int t = decltype(Tc)::value;
        constexpr int dy = t / 3, dx = t % 3;
        // (kk: 32 pixels further = 32 / W image rows, or 32 columns at W = 64)
        constexpr int roff = ((dy + kk * 32 / W) * HW2 + (kk * 32) % W) * RS;
        constexpr int fl = (W == 8 && (dy & 1)) ? 1 : 0;
        o[0] = tr_read<roff>(ba[fl][dx][0]);
        o[1] = tr_read<roff>(ba[fl][dx][1]);
      };
      read_b(ic<0>{}, fb[0]);
      auto tap = [&](auto Tc) __attribute__((always_inline)) {
        constexpr int t = decltype(Tc)::value;
        if constexpr (t + 1 < 9) {
          read_b(ic<t + 1>{}, fb[(t + 1) & 1]);
          asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        asm volatile("" : "+v"(fb[t & 1][0]), "+v"(fb[t & 1][1]));
        if (t == 0) {
#pragma unroll
          for (int i = 0; i < MA; ++i) asm volatile("" : "+v"(fa[i][0]), "+v"(fa[i][1]));
        }
        const bf16x8 b = __builtin_bit_cast(bf16x8, __builtin_shufflevector(fb[t & 1][0], fb[t & 1][1], 0, 1, 2, 3, 4, 5, 6, 7));
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < MA; ++i) {
          const bf16x8 av = __builtin_bit_cast(bf16x8, __builtin_shufflevector(fa[i][0], fa[i][1], 0, 1, 2, 3, 4, 5, 6, 7));
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b, acc[i][t], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
      };
      tap(ic<0>{}); tap(ic<1>{}); tap(ic<2>{}); tap(ic<3>{}); tap(ic<4>{});
      tap(ic<5>{}); tap(ic<6>{}); tap(ic<7>{}); tap(ic<8>{});
    };
    kloop(ic<0>{});
    kloop(ic<1>{});
  };
  // ---- the stage loop: NSTG buffers, stage s + NSTG - 1 in flight while s
  // computes; per stage every wave issues exactly NI pieces, so "stage s
  // landed" is vmcnt <= NI x (stages issued after s) ----
  const int nst = send - sbeg;
  if (nst > 0) issue(sbeg, 0);
  if (NSTG == 3 && nst > 1) issue(sbeg + 1, 1);
  for (int s = 0; s < nst; ++s) {
    if (NSTG == 3 && s + 1 < nst) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(NI) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    // (after the barrier every wave is past compute(s - 1): its buffer is free)
    if (s + NSTG - 1 < nst) issue(sbeg + s + NSTG - 1, (s + NSTG - 1) % NSTG);
    compute(s % NSTG);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  constexpr int MB = 1;
  const int wa = 0;

  // partial[split][a / 4][tap][b][a % 4]: the accumulator's own layout (a
  // lane holds 4 consecutive dy channels of one x channel), one 16-B store
  // per lane and (i, j, tap), 16 lanes = 256 contiguous bytes -- 36 dwordx4
  // stores per wave instead of 144 dword ones into 64-B pieces
  // (rr_wgrad_reduce maps the layout back: launch_reduce's alayout)
#pragma unroll
  for (int i = 0; i < MA; ++i) {
    const int b = b0 + wb * 16 * MB + gi;
    const int a4 = (a0 + wa * 16 * MA + i * 16) / 4 + g;
#pragma unroll
    for (int t = 0; t < 9; ++t)
      *reinterpret_cast<f32x4 *>(a.partial + ((((long long)split * (a.CA / 4) + a4) * 9 + t) * a.CB + b) * 4) =
          acc[i][t];
  }
}

// dw[(a*CB + b)*taps + t] (+)= sum_s partial[s][a][t][b]   (fixed order, 4 chains)
__global__ void wgrad_reduce(const float *__restrict__ partial, float *__restrict__ dw,
                             int CA, int CB, int taps, int nsplit, int accumulate) {
  const long long total = (long long)CA * CB * taps;
  const long long slab = total;
  for (long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x; o < total;
       o += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(o % CB);
    const long long at = o / CB;
    const int t = (int)(at % taps);
    const int ar = (int)(at / taps);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int sp = 0;
    for (; sp + 4 <= nsplit; sp += 4) {
      s0 += partial[(sp + 0) * slab + o];
      s1 += partial[(sp + 1) * slab + o];
      s2 += partial[(sp + 2) * slab + o];
      s3 += partial[(sp + 3) * slab + o];
    }
    for (; sp < nsplit; ++sp) s0 += partial[sp * slab + o];
    const float s = (s0 + s1) + (s2 + s3);
    const long long di = ((long long)ar * CB + b) * taps + t;
    dw[di] = accumulate ? dw[di] + s : s;
  }
}

// Split-parallel variant: G split groups x (256/G) float4 output columns per
// block; group g sums splits g, g+G, ... and the groups are combined in LDS in
// fixed order (deterministic).  Needs slab % 4 == 0.
// alayout 1: the slabs are [a / 4][tap][b][a % 4] (wgrad3_halo_kernel, and
// wgrad_kernel where CA % 4 == 0), 0: [a][tap][b]; the split sum is
// elementwise either way (same order)
template <int G>
__global__ __launch_bounds__(256) void wgrad_reduce_g(const float *__restrict__ partial,
                                                       float *__restrict__ dw, int CA, int CB,
                                                       int taps, int nsplit, int accumulate, int alayout) {
  constexpr int NC = 256 / G;                  // float4 columns per block
  __shared__ float4 red[G][NC];
  const long long slab = (long long)CA * CB * taps;
  const int col = threadIdx.x % NC, g = threadIdx.x / NC;
  const long long o4 = (long long)blockIdx.x * NC + col;
  const bool live = o4 * 4 < slab;
  const float4 *p4 = reinterpret_cast<const float4 *>(partial);
  const long long s4 = slab / 4;
  float4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  if (live) {
    int sp = g;
    for (; sp + G < nsplit; sp += 2 * G) {
      const float4 u = p4[sp * s4 + o4], v = p4[(sp + G) * s4 + o4];
      s0.x += u.x; s0.y += u.y; s0.z += u.z; s0.w += u.w;
      s1.x += v.x; s1.y += v.y; s1.z += v.z; s1.w += v.w;
    }
    if (sp < nsplit) {
      const float4 u = p4[sp * s4 + o4];
      s0.x += u.x; s0.y += u.y; s0.z += u.z; s0.w += u.w;
    }
  }
  red[g][col] = float4{s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w};
  __syncthreads();
  if (g != 0 || !live) return;
  float4 s = red[0][col];
#pragma unroll
  for (int i = 1; i < G; ++i) {
    const float4 u = red[i][col];
    s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
  }
  const float v[4] = {s.x, s.y, s.z, s.w};
  if (alayout) {
    const int b = (int)(o4 % CB);
    const long long at = o4 / CB;
    const int t = (int)(at % taps);
    const int a4 = (int)(at / taps);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long di = ((long long)(a4 * 4 + e) * CB + b) * taps + t;
      dw[di] = accumulate ? dw[di] + v[e] : v[e];
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long long o = o4 * 4 + e;
    const int b = (int)(o % CB);
    const long long at = o / CB;
    const int t = (int)(at % taps);
    const int ar = (int)(at / taps);
    const long long di = ((long long)ar * CB + b) * taps + t;
    dw[di] = accumulate ? dw[di] + v[e] : v[e];
  }
}

static void launch_reduce(const float *ws, float *dw, int CA, int CB, int taps, int nsplit,
                          int accumulate, int alayout, hipStream_t st) {
  const long long total = (long long)CA * CB * taps;
  if (total % 4) {
    hipLaunchKernelGGL(wgrad_reduce, dim3(rr_grid_cap((total + 255) / 256, 8192)), dim3(256), 0, st,
                       ws, dw, CA, CB, taps, nsplit, accumulate);
    return;
  }
  // smallest G (fewest LDS combines) that still gives >= ~1024 blocks
  int G = 1;
  while (G < 16 && G * 2 <= nsplit && (total / 4 + 256 / G - 1) / (256 / G) < 1024) G *= 2;
  const unsigned nb = (unsigned)((total / 4 + 256 / G - 1) / (256 / G));
  switch (G) {
    case 1: hipLaunchKernelGGL(wgrad_reduce_g<1>, dim3(nb), dim3(256), 0, st, ws, dw, CA, CB, taps, nsplit, accumulate, alayout); break;
    case 2: hipLaunchKernelGGL(wgrad_reduce_g<2>, dim3(nb), dim3(256), 0, st, ws, dw, CA, CB, taps, nsplit, accumulate, alayout); break;
    case 4: hipLaunchKernelGGL(wgrad_reduce_g<4>, dim3(nb), dim3(256), 0, st, ws, dw, CA, CB, taps, nsplit, accumulate, alayout); break;
    case 8: hipLaunchKernelGGL(wgrad_reduce_g<8>, dim3(nb), dim3(256), 0, st, ws, dw, CA, CB, taps, nsplit, accumulate, alayout); break;
    default: hipLaunchKernelGGL(wgrad_reduce_g<16>, dim3(nb), dim3(256), 0, st, ws, dw, CA, CB, taps, nsplit, accumulate, alayout); break;
  }
}

struct Plan {
  int BA, BB, nsplit, split_len, nablk, nbblk, taps, CA, CB;
};

Plan plan_of(const rr_wgrad_desc *d) {
  Plan p;
  p.taps = d->mode == RR_CONV3X3 ? 9 : (d->mode == RR_CONVT_UP ? 4 : 1);
  const bool convT = d->mode == RR_CONVT_UP;
  p.CA = convT ? d->c_in1 : d->c_out;
  p.CB = convT ? d->c_out : d->c_in1 + d->c_in2;
  const int c1 = convT ? d->c_out : d->c_in1;
  const int c2 = convT ? 0 : d->c_in2;
  p.BA = (p.CA % 128 == 0) ? 128 : 64;
  p.BB = (p.CB % 128 == 0 && c1 % 128 == 0 && c2 % 128 == 0) ? 128 : 64;
  p.nablk = (p.CA + p.BA - 1) / p.BA;
  p.nbblk = (p.CB + p.BB - 1) / p.BB;
  const long long P = (long long)d->n * d->h * d->w;
  const long long tiles = (long long)p.nablk * p.nbblk * p.taps;
  // ~1024 workgroups; ~512 for the bf16 1x1 / convT weight grads whose split
  // partials (nsplit x the weight, written and read back in fp32) would be
  // more than an eighth of the activation bytes at 1024 -- on the 16x16 /
  // 8x8 maps they moved more bytes than the activations (1x1 / convT layers
  // 10-30 % faster at 512, r6h); elsewhere 512 lost parallelism (up1, dec2.sc)
  auto split_len = [&](long long target) {
    const long long want = (target + tiles - 1) / tiles;
    const long long maxs = (P + 4 * BKP_PLAN - 1) / (4 * BKP_PLAN);   // >= 4 stages per split
    long long ns = want < maxs ? want : maxs;
    if (ns < 1) ns = 1;
    long long len = (P + ns - 1) / ns;
    return (len + BKP_PLAN - 1) / BKP_PLAN * BKP_PLAN;
  };
  long long len = split_len(1024);
  if (d->dtype == RR_BF16 && d->mode != RR_CONV3X3) {
    const long long part = (P + len - 1) / len * p.CA * p.CB * p.taps * 4;
    const long long act = 2 * P * (convT ? d->c_in1 + 4LL * d->c_out : (long long)d->c_out + d->c_in1 + d->c_in2);
    if (8 * part > act) len = split_len(512);
  }
  p.split_len = (int)len;
  p.nsplit = (int)((P + len - 1) / len);
  return p;
}

template <typename T, int BA, int BB>
int launch(const rr_wgrad_desc *d, const Plan &pl, WgradArgs &a, hipStream_t st) {
  const long long nblk = (long long)pl.nablk * pl.nbblk * pl.taps * pl.nsplit;
  dim3 grid((unsigned)nblk), block(256);
  switch (d->mode) {
    case RR_CONV3X3: hipLaunchKernelGGL((wgrad_kernel<T, BA, BB, RR_CONV3X3>), grid, block, 0, st, a); break;
    case RR_CONV1X1: hipLaunchKernelGGL((wgrad_kernel<T, BA, BB, RR_CONV1X1>), grid, block, 0, st, a); break;
    case RR_CONVT_UP: hipLaunchKernelGGL((wgrad_kernel<T, BA, BB, RR_CONVT_UP>), grid, block, 0, st, a); break;
    default: return RR_EINVAL;
  }
  RR_CHECK_LAUNCH();
  return RR_OK;
}

template <typename T>
int launch_t(const rr_wgrad_desc *d, const Plan &pl, WgradArgs &a, hipStream_t st) {
  if (pl.BA == 128 && pl.BB == 128) return launch<T, 128, 128>(d, pl, a, st);
  if (pl.BA == 128) return launch<T, 128, 64>(d, pl, a, st);
  if (pl.BB == 128) return launch<T, 64, 128>(d, pl, a, st);
  return launch<T, 64, 64>(d, pl, a, st);
}

}  // namespace

static bool halo_ok(const rr_wgrad_desc *d) {
  if (d->dtype != RR_BF16 || d->mode != RR_CONV3X3) return false;
  if (!(d->w == 8 || d->w == 16 || d->w == 32 || d->w == 64)) return false;
  if (d->h % (64 / d->w)) return false;
  if (d->c_out % 64 || d->c_in1 % 64 || d->c_in2 % 64) return false;
  return rr_path("wgrad_halo", 1) != 0;   // RR_PATH wgrad_halo=0: the tiled kernel (tests)
}

struct HaloPlan { int stages, split_stages, nsplit; };

static HaloPlan halo_plan(const rr_wgrad_desc *d) {
  HaloPlan p;
  const long long P = (long long)d->n * d->h * d->w;
  p.stages = (int)(P / 64);
  const int tiles = (d->c_out / 64) * ((d->c_in1 + d->c_in2) / 64);
  // ~512 workgroups (one full wave at 2 blocks/CU, measured best: 256 and
  // 1024 were 2.5 % / 1.5 % slower on the step, r5y / r5zc)
  const int target = 512;
  int want = (target + tiles - 1) / tiles;
  int maxs = (p.stages + 3) / 4;                    // >= 4 stages per split
  int ns = want < maxs ? want : maxs;
  if (ns < 1) ns = 1;
  p.split_stages = (p.stages + ns - 1) / ns;
  p.nsplit = (p.stages + p.split_stages - 1) / p.split_stages;
  return p;
}

extern "C" size_t rr_wgrad_workspace(const rr_wgrad_desc *d) {
  if (!d) return 0;
  if (swgrad_ok(d))
    return (size_t)swgrad_nsplit(d) * d->c_out * 9 * (d->c_in1 + d->c_in2) * sizeof(float);
  if (halo_ok(d)) {
    const HaloPlan hp = halo_plan(d);
    return (size_t)hp.nsplit * d->c_out * 9 * (d->c_in1 + d->c_in2) * sizeof(float);
  }
  const Plan p = plan_of(d);
  return (size_t)p.nsplit * p.CA * p.taps * p.CB * sizeof(float);
}

// the weight-grad kernel rr_wgrad would launch for *d (same decisions;
// static strings, never NULL)
extern "C" const char *rr_wgrad_kernel_name(const rr_wgrad_desc *d) {
  if (!d) return "invalid";
  if (swgrad_ok(d)) return d->w == 64 ? "swgrad_kernel<64>" : "swgrad_kernel<32>";
  if (halo_ok(d)) {
    switch (d->w) {
      case 64: return "wgrad3_halo_kernel<64>";
      case 32: return "wgrad3_halo_kernel<32>";
      case 16: return "wgrad3_halo_kernel<16>";
      default: return "wgrad3_halo_kernel<8>";
    }
  }
  const Plan pl = plan_of(d);
  static const char *tn[2][2][2][4] = {
      {{{"wgrad_kernel<f32,64,64,m0>", "wgrad_kernel<f32,64,64,m1>", "wgrad_kernel<f32,64,64,m2>", "wgrad_kernel<f32,64,64,m3>"},
        {"wgrad_kernel<f32,64,128,m0>", "wgrad_kernel<f32,64,128,m1>", "wgrad_kernel<f32,64,128,m2>", "wgrad_kernel<f32,64,128,m3>"}},
       {{"wgrad_kernel<f32,128,64,m0>", "wgrad_kernel<f32,128,64,m1>", "wgrad_kernel<f32,128,64,m2>", "wgrad_kernel<f32,128,64,m3>"},
        {"wgrad_kernel<f32,128,128,m0>", "wgrad_kernel<f32,128,128,m1>", "wgrad_kernel<f32,128,128,m2>", "wgrad_kernel<f32,128,128,m3>"}}},
      {{{"wgrad_kernel<bf16,64,64,m0>", "wgrad_kernel<bf16,64,64,m1>", "wgrad_kernel<bf16,64,64,m2>", "wgrad_kernel<bf16,64,64,m3>"},
        {"wgrad_kernel<bf16,64,128,m0>", "wgrad_kernel<bf16,64,128,m1>", "wgrad_kernel<bf16,64,128,m2>", "wgrad_kernel<bf16,64,128,m3>"}},
       {{"wgrad_kernel<bf16,128,64,m0>", "wgrad_kernel<bf16,128,64,m1>", "wgrad_kernel<bf16,128,64,m2>", "wgrad_kernel<bf16,128,64,m3>"},
        {"wgrad_kernel<bf16,128,128,m0>", "wgrad_kernel<bf16,128,128,m1>", "wgrad_kernel<bf16,128,128,m2>", "wgrad_kernel<bf16,128,128,m3>"}}}};
  const int mi = d->mode >= 0 && d->mode <= 3 ? d->mode : 0;
  return tn[d->dtype == RR_BF16][pl.BA == 128][pl.BB == 128][mi];
}

// the reduce of *d's split partials: (CA, CB, taps, nsplit) of the slab
static void reduce_shape(const rr_wgrad_desc *d, int &CA, int &CB, int &taps, int &nsplit) {
  if (swgrad_ok(d)) {
    CA = d->c_out; CB = d->c_in1 + d->c_in2; taps = 9; nsplit = swgrad_nsplit(d);
  } else if (halo_ok(d)) {
    CA = d->c_out; CB = d->c_in1 + d->c_in2; taps = 9; nsplit = halo_plan(d).nsplit;
  } else {
    const Plan pl = plan_of(d);
    CA = pl.CA; CB = pl.CB; taps = pl.taps; nsplit = pl.nsplit;
  }
}

static bool wgrad_desc_ok(const rr_wgrad_desc *d) {
  return d->mode == RR_CONV3X3 || d->mode == RR_CONV1X1 || d->mode == RR_CONVT_UP;
}

extern "C" int rr_wgrad_reduce(const rr_wgrad_desc *d, const void *ws, size_t ws_bytes, float *dw,
                               rr_stream stream) {
  if (!d || !ws || !dw || !wgrad_desc_ok(d)) return RR_EINVAL;
  if (d->c_in1 % 64 || d->c_in2 % 64 || d->c_out % 64) return RR_EUNSUPPORTED;
  if (ws_bytes < rr_wgrad_workspace(d)) return RR_EWORKSPACE;
  int CA, CB, taps, nsplit;
  reduce_shape(d, CA, CB, taps, nsplit);
  const int alayout = !swgrad_ok(d) && CA % 4 == 0;   // the halo / tiled kernels' slab layout
  launch_reduce((const float *)ws, dw, CA, CB, taps, nsplit, d->accumulate, alayout, (hipStream_t)stream);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" int rr_wgrad(const rr_wgrad_desc *d, const void *dy, const void *x1,
                        const void *x2, float *dw, void *ws, size_t ws_bytes,
                        rr_stream stream) {
  if (!dw) return RR_EINVAL;
  const int rc = rr_wgrad_partial(d, dy, x1, x2, ws, ws_bytes, stream);
  if (rc) return rc;
  return rr_wgrad_reduce(d, ws, ws_bytes, dw, stream);
}

extern "C" int rr_wgrad_pre_ok(const rr_wgrad_desc *d) {
  return d && d->mode == RR_CONV3X3 && !d->c_in2 && !d->accumulate && swgrad_ok(d) ? 1 : 0;
}

// conv2's weight grad with BN1 + PReLU of its input folded in: x1 is t1 and
// the kernel reads PReLU(t1 * pre_scale + pre_shift) (the bytes
// rr_affine_act(t1, pre_scale, pre_shift, pre_alpha) would store); the
// partial slabs then go through rr_wgrad_reduce
extern "C" int rr_wgrad_pre(const rr_wgrad_desc *d, const void *dy, const void *x1,
                            const float *pre_scale, const float *pre_shift, const float *pre_alpha,
                            float *dw, void *ws, size_t ws_bytes, rr_stream stream) {
  if (!d || !dy || !x1 || !dw || !pre_scale || !pre_shift || !pre_alpha) return RR_EINVAL;
  if (!rr_wgrad_pre_ok(d)) return RR_EUNSUPPORTED;
  const size_t need = rr_wgrad_workspace(d);
  if (!ws || ws_bytes < need) return RR_EWORKSPACE;
  const int rc = swgrad_launch_pre(d, dy, x1, pre_scale, pre_shift, pre_alpha, ws, (hipStream_t)stream);
  if (rc) return rc;
  return rr_wgrad_reduce(d, ws, ws_bytes, dw, stream);
}

extern "C" int rr_wgrad_partial(const rr_wgrad_desc *d, const void *dy, const void *x1,
                                const void *x2, void *ws, size_t ws_bytes, rr_stream stream) {
  if (!d || !dy || !x1) return RR_EINVAL;
  if (d->mode != RR_CONV3X3 && d->mode != RR_CONV1X1 && d->mode != RR_CONVT_UP) return RR_EINVAL;
  if (d->c_in1 % 64 || d->c_in2 % 64 || d->c_out % 64) return RR_EUNSUPPORTED;
  if (d->c_in2 > 0 && (!x2 || d->mode == RR_CONVT_UP)) return RR_EINVAL;
  const long long P = (long long)d->n * d->h * d->w;
  if (P <= 0 || P * 4 > 0x7fffffffLL) return RR_EUNSUPPORTED;
  const Plan pl = plan_of(d);
  const size_t need = rr_wgrad_workspace(d);
  if (!ws || ws_bytes < need) return RR_EWORKSPACE;
  WgradArgs a;
  const bool convT = d->mode == RR_CONVT_UP;
  a.A = (const char *)(convT ? x1 : dy);
  a.B1 = (const char *)(convT ? dy : x1);
  a.B2 = (const char *)(convT ? nullptr : x2);
  a.partial = (float *)ws;
  a.CA = pl.CA; a.CB = pl.CB;
  a.c1 = convT ? d->c_out : d->c_in1;
  a.c2 = convT ? 0 : d->c_in2;
  a.taps = pl.taps;
  a.n = d->n; a.h = d->h; a.w = d->w;
  a.P = (int)P;
  a.split_len = pl.split_len;
  a.nablk = pl.nablk; a.nbblk = pl.nbblk;
  a.xcd = 1;                                   // XCD-aware workgroup order
  a.fd_w = make_fastdiv((uint32_t)d->w);
  a.fd_hw = make_fastdiv((uint32_t)(d->h * d->w));
  hipStream_t st = (hipStream_t)stream;
  if (swgrad_ok(d)) {
    const int rc = swgrad_launch(d, dy, x1, x2, ws, st);
    if (rc) return rc;
    RR_CHECK_LAUNCH();
    return RR_OK;
  }
  if (halo_ok(d)) {
    const HaloPlan hp = halo_plan(d);
    Halo3Args ha;
    ha.A = (const char *)dy; ha.B1 = (const char *)x1; ha.B2 = (const char *)x2;
    ha.partial = (float *)ws;
    ha.CA = d->c_out; ha.CB = d->c_in1 + d->c_in2; ha.c1 = d->c_in1; ha.c2 = d->c_in2;
    ha.n = d->n; ha.h = d->h; ha.w = d->w;
    ha.lw = __builtin_ctz((unsigned)d->w);
    ha.stages = hp.stages; ha.split_stages = hp.split_stages;
    ha.nablk = ha.CA / 64; ha.nbblk = ha.CB / 64;
    ha.xcd = a.xcd;
    const dim3 grid((unsigned)(ha.nablk * ha.nbblk * hp.nsplit)), block(256);
    switch (d->w) {
      case 64: hipLaunchKernelGGL((wgrad3_halo_kernel<64>), grid, block, 0, st, ha); break;
      case 32: hipLaunchKernelGGL((wgrad3_halo_kernel<32>), grid, block, 0, st, ha); break;
      case 16: hipLaunchKernelGGL((wgrad3_halo_kernel<16>), grid, block, 0, st, ha); break;
      default: hipLaunchKernelGGL((wgrad3_halo_kernel<8>), grid, block, 0, st, ha); break;
    }
    RR_CHECK_LAUNCH();
    return RR_OK;
  }
  return d->dtype == RR_BF16 ? launch_t<bf16_t>(d, pl, a, st) : launch_t<float>(d, pl, a, st);
}
