// swgrad.hip -- row-streaming 3x3 bf16 weight gradient for the wide layers
// (64 x 64 and 32 x 32 maps) whose output gradient has 64 or 128 channels:
// res1, res2, dec1 and dec2 conv1 / conv2 of ResUNet (14_train_unified_advanced.py:96-115,
// 151-186), concat inputs of up to 192 channels.  A 128-channel dy is read as
// two 64-channel slices: a workgroup owns one (dy slice, input slice) pair.
//
//   dW[co][tap][ci] = sum_p dy[p][co] * x[p + tap][ci]
//
// Like stream3.hip: one persistent 512-thread workgroup per CU walks a
// contiguous range of output rows in 128-pixel steps.  Per step one LDS-DMA
// batch brings the step's NEW input rows into a ring of zero-haloed rows
// (every input row is read once) and the step's 128 x 64 dy tile into a
// 4-tile ring, D = 2 steps ahead of the MFMAs.  The workgroup owns one
// 64-channel slice of the input (concat inputs: 2 or 3 slices) and of dy, and
// accumulates the whole 64 x 576 dW block in registers over all its pixels;
// the per-workgroup partial slabs are summed by rr_wgrad's fixed-order
// reduce (deterministic, no float atomics).
//
// Instruction budget is what bounds this kernel (the scalar unit is shared by
// the CU's 8 waves): the ring holds exactly 4 steps (4 row segments of RPS
// rows, 4 dy tiles) and the step loop is unrolled by 4, so every LDS address
// is a loop-invariant lane VGPR plus an immediate offset, and a DMA piece
// costs a handful of scalar ops.  The two halo columns of every ring row are
// zeroed once and never written by the DMA; rows outside the image come from
// a zero buffer.
//
// MFMA (16x16x32 bf16): A = dy^T (16 output channels x 32 pixels), B = x
// shifted by the tap (32 pixels x 16 input channels); both read with
// ds_read_b64_tr_b16 (4 pixels x 16 channels -> lane = channel).  Both LDS
// images are pixel-major, 128 B a pixel, 16-B chunk c of pixel p stored at
// slot c ^ swz(p): a transposed read's 32-lane half touches 8 pixels {P..P+3,
// P+8..P+11} (or the +4 set) x one aligned chunk pair; swz(p) = 2 * {0,1,2,3,
// 2,3,0,1}[p/2 % 8] gives the 4 pixels of each parity distinct chunk pairs for
// P = 0, 1, 2 (mod 16) -- the dy tile's offset and the three tap columns -- so
// all 64 banks are hit once.  Row strides are multiples of 256 B.  The
// source-side half of the swizzle is in the DMA addresses (LDS-DMA writes
// lane-linear 1-KB pieces).
//
// Waves: 2 (32 output channels) x 4 (16 input channels); a step is 36 groups
// (32-pixel slice kk, tap t) of one B fragment and two MFMAs.
//
// vmcnt: every step issues exactly DMAW DMA instructions per wave and no other
// vector-memory op, so DMA(v) is retired by vmcnt((D - 1) DMAW).
#include "common.h"
#include "swgrad.h"

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace {

constexpr int SW_WG = 256;
constexpr int SW_D = 2;                         // steps of prefetch in flight
constexpr int SW_PF = 2;                        // groups of LDS reads in flight (2: 146 vs 154 us for 4 at W=64)

__host__ __device__ constexpr int sw_swz(int p) { return 2 * ((0x10323210u >> (4 * ((p >> 1) & 7))) & 0xf); }

template <int W> struct SWGeo {
  static constexpr int RPS = 128 / W;                      // image rows per 128-pixel step
  static constexpr int RPX = W + 2;                        // zero halo column either side
  static constexpr int ROWB = RPX * 128;
  static constexpr int RING = 4 * RPS;                     // 4 row segments
  static constexpr int DYB = 128 * 128;                    // dy tile of a step
  static constexpr int DYOFF = RING * ROWB;
  static constexpr int XPC = RPS * W / 8;                  // x pieces per step (8 pixels)
  static constexpr int DMAW = (XPC + DYB / 1024) / 8;      // DMA pieces per wave per step
  static constexpr int LDS = DYOFF + 4 * DYB;
  static_assert(XPC % 8 == 0 && (DYB / 1024) % 8 == 0, "pieces split over 8 waves");
  static_assert(ROWB % 256 == 0, "bank-aligned rows");
  static_assert((RING - 1) * ROWB + (W - 32) * 128 < 65536, "B read offsets are 16-bit immediates");
  static_assert(RING >= (SW_D + 1) * RPS + 2, "ring");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// source of rows outside the image (largest lane offset: 63 px x 384 B + 112)
__device__ __attribute__((aligned(16))) const char sw_zero[32768] = {0};

enum { SW_PRE = 0, SW_COMP = 1 };
struct SwCur { int kind, n, y0, c; };

typedef short s16x4v __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// transposed LDS read as inline asm: with LDS-DMA in flight hipcc would put a
// vmcnt(0) before every visible LDS read; completion is counted by sw_lgkm
#define SW_TRD(r, addr, off) \
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(off))

#define SW_LG(n) \
  case n: asm volatile("s_waitcnt lgkmcnt(" #n ")" ::: "memory"); break;
__device__ __forceinline__ void sw_lgkm(int n) {   // n folds to a constant after unrolling
  switch (n) {
    SW_LG(0) SW_LG(1) SW_LG(2) SW_LG(3) SW_LG(4) SW_LG(5) SW_LG(6) SW_LG(7) SW_LG(8)
    SW_LG(9) SW_LG(10) SW_LG(11) SW_LG(12) SW_LG(13) SW_LG(14) SW_LG(15)
    default: asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); break;
  }
}

// PRE: x1 is the pre-BN t1; every input row that lands in the ring becomes
// a1 = PReLU(t1 * s + b) in LDS (rr_affine_act's fp32 expression and bf16
// rounding) before any group reads it -- BN1 + PReLU folded into conv2's
// weight grad (14:101-104), the a1 tensor never stored
template <int W, bool PRE>
__global__ __launch_bounds__(512, 2) void swgrad_kernel(SWArgs a) {
  using G = SWGeo<W>;
  constexpr int RPS = G::RPS, ROWB = G::ROWB, RING = G::RING, DYB = G::DYB, DYOFF = G::DYOFF;
  constexpr int XPC = G::XPC, DMAW = G::DMAW, D = SW_D, PF = SW_PF;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wv & 1, wk = wv >> 1;          // output channels 32 wc.., input channels 16 wk..
  const int H = a.h;
  const int spi = H / RPS;
  // workgroup -> (dy slice ds, input slice, pixel range r)
  const int nxs = (a.c1 + a.c2) / 64;
  const int sq = blockIdx.x / a.nwg_ps, r = blockIdx.x - sq * a.nwg_ps;
  const int ds = sq / nxs, slice = sq - ds * nxs;
  const int dys = a.cout * 2;                              // bytes per dy pixel
  const int cbeg = (int)((long long)r * a.nsteps / a.nwg_ps);
  const int cend = (int)((long long)(r + 1) * a.nsteps / a.nwg_ps);
  const int ci0 = slice * 64;
  const bool first = ci0 < a.c1;
  const char *const xsrc = (first ? a.x1 : a.x2) + (first ? ci0 : ci0 - a.c1) * 2;
  const int xpb = (first ? a.c1 : a.c2) * 2;              // bytes per source pixel

  // ---- halo columns: zeroed once, never written by the DMA ----
  for (int u = tid; u < RING * 16; u += 512) {
    const int row = u >> 4, side = (u >> 3) & 1, c = u & 7;
    *reinterpret_cast<uint4 *>(smem + row * ROWB + (side ? (W + 1) * 128 : 0) + c * 16) = uint4{0, 0, 0, 0};
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // ---- DMA pieces (piece i * 8 + wave of a step; i < XPC / 8: x rows) ----
  // x piece: ring row rr of the step, pixels 8 j .. 8 j + 7 (LDS px 1 + 8 j ..)
  // dy piece: tile pixels 8 t .. 8 t + 7
  uint32_t pofs[DMAW];                          // lane source offset (loop-invariant)
  int prow[DMAW], pdst[DMAW];                   // uniform: ring row, LDS offset in the segment / tile
#pragma unroll
  for (int i = 0; i < DMAW; ++i) {
    const int t = i * 8 + wv;
    if (i < XPC / 8) {
      const int rr = t / (W / 8), j = t % (W / 8);
      const int px = 1 + 8 * j + (lane >> 3), chunk = (lane & 7) ^ sw_swz(px & 15);
      prow[i] = rr;
      pdst[i] = rr * ROWB + (1 + 8 * j) * 128;
      pofs[i] = (uint32_t)((px - 1) * xpb + chunk * 16);
    } else {
      const int tt = t - XPC;
      const int p = 8 * tt + (lane >> 3), chunk = (lane & 7) ^ sw_swz(p & 15);
      prow[i] = 0;
      pdst[i] = tt * 1024;
      pofs[i] = (uint32_t)(p * dys + ds * 128 + chunk * 16);
    }
  }
  const long long xrow_b = (long long)W * xpb;             // bytes per image row of the source
  // issue piece i of the step at cursor cu into segment / tile seg
  auto issue_piece = [&](int i, int seg, const SwCur &cu, bool live) __attribute__((always_inline)) {
    asm volatile("" : "+v"(pofs[i]));
    if (i < XPC / 8) {
      const int y0 = cu.kind == SW_PRE ? cu.y0 - RPS + 1 : cu.y0 + 1;
      const int y = y0 + prow[i];
      const bool ok = live & ((unsigned)y < (unsigned)H);
      const char *base = ok ? xsrc + (long long)(cu.n * H + y) * xrow_b : sw_zero;
      __builtin_amdgcn_global_load_lds((const void *)(base + pofs[i]),
                                       LDS_PTR(smem + seg * RPS * ROWB + pdst[i]), 16, 0, 0);
    } else {
      const char *base = live ? a.dy + (long long)(cu.n * H + cu.y0) * W * dys : a.dy;
      __builtin_amdgcn_global_load_lds((const void *)(base + pofs[i]),
                                       LDS_PTR(smem + DYOFF + seg * DYB + pdst[i]), 16, 0, 0);
    }
  };
  auto advance = [&](SwCur &cu) __attribute__((always_inline)) {
    if (cu.kind == SW_PRE) {
      cu.kind = SW_COMP;
    } else {
      ++cu.c;
      cu.y0 += RPS;
      if (cu.y0 == H) { cu.y0 = 0; ++cu.n; cu.kind = SW_PRE; }
    }
  };

  // ---- lane parts of the transposed reads ----
  // lane = 16 g + 4 q + pp reads pixel 8 g + q (+ 4 for the second half) at
  // channels 4 pp .. 4 pp + 3 of a 16-channel block (chunks 2 cb, 2 cb + 1)
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  auto lofs = [&](int P, int cb) __attribute__((always_inline)) {
    return (uint32_t)(P * 128 + (((2 * cb) ^ sw_swz(P & 15)) + (pp >> 1)) * 16 + (pp & 1) * 8);
  };
  const uint32_t sbase = (uint32_t)(uintptr_t)smem;
  uint32_t la[2][2], lb[3][2];                  // dy: [m][half]; x: [tap column][half]
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int m = 0; m < 2; ++m) la[m][h] = sbase + DYOFF + lofs(8 * g + q + 4 * h, 2 * wc + m);
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) lb[dx][h] = sbase + lofs(dx + 8 * g + q + 4 * h, wk);
  }

  // PRE: a thread transforms chunks tid + 512 j of a step's input rows, all at
  // one ring-row pixel and 16-B slot: its 8 channels' (s, b) in registers
  f32x4 pcs[PRE ? 2 : 1], pcb[PRE ? 2 : 1];
  float palp = 0.f;
  if constexpr (PRE) {
    const int rem = tid % (W * 8);
    const int px = 1 + (rem >> 3), c = (rem & 7) ^ sw_swz(px & 15);
    pcs[0] = *reinterpret_cast<const f32x4 *>(a.pre_s + ci0 + 8 * c);
    pcs[1] = *reinterpret_cast<const f32x4 *>(a.pre_s + ci0 + 8 * c + 4);
    pcb[0] = *reinterpret_cast<const f32x4 *>(a.pre_b + ci0 + 8 * c);
    pcb[1] = *reinterpret_cast<const f32x4 *>(a.pre_b + ci0 + 8 * c + 4);
    palp = a.pre_alpha[0];
    __builtin_amdgcn_s_waitcnt(0x0F70);        // vmcnt(0): resident before any DMA is in flight
  }

  f32x4 acc[2][9];                              // [co block m][tap]
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  SwCur ld;
  ld.c = cbeg;
  ld.n = cbeg / spi;
  ld.y0 = (cbeg - ld.n * spi) * RPS;
  ld.kind = SW_PRE;
  SwCur cp = ld;
#pragma unroll
  for (int k = 0; k < D; ++k) {
#pragma unroll
    for (int i = 0; i < DMAW; ++i) issue_piece(i, k, ld, ld.c < cend);
    advance(ld);
  }

  // one step; U = step index mod 4 (ring segment and dy tile of the step)
  auto step = [&](auto Uc) __attribute__((always_inline)) {
    constexpr int U = decltype(Uc)::value;
    constexpr int LSEG = (U + D) & 3;           // segment / tile of the step loaded now
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((D - 1) * DMAW) : "memory");
    if constexpr (PRE) {
      // the step's input rows (segment U): a compute step's image rows
      // y0 + 1 + r, a pre-load's y0 - 1 and y0 (the rows it reads)
      constexpr int NCH = RPS * W * 8;
      static_assert(NCH % 512 == 0, "whole chunks per thread");
      const bool comp = cp.kind == SW_COMP;
#pragma unroll
      for (int j = 0; j < NCH / 512; ++j) {
        const int k = tid + 512 * j;
        const int r = k / (W * 8), rem = k - r * (W * 8);
        const int px = 1 + (rem >> 3);
        const int y = comp ? cp.y0 + 1 + r : cp.y0 - RPS + 1 + r;
        if (y < 0 || y >= H || (!comp && r < RPS - 2)) continue;
        const uint32_t addr = sbase + (U * RPS + r) * ROWB + px * 128 + (rem & 7) * 16;
        i32x4 v;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
        f32x4 lo = f32x4{__uint_as_float((uint32_t)v[0] << 16), __uint_as_float((uint32_t)v[0] & 0xffff0000u),
                         __uint_as_float((uint32_t)v[1] << 16), __uint_as_float((uint32_t)v[1] & 0xffff0000u)};
        f32x4 hi = f32x4{__uint_as_float((uint32_t)v[2] << 16), __uint_as_float((uint32_t)v[2] & 0xffff0000u),
                         __uint_as_float((uint32_t)v[3] << 16), __uint_as_float((uint32_t)v[3] & 0xffff0000u)};
        lo = lo * pcs[0] + pcb[0];
        hi = hi * pcs[1] + pcb[1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          lo[e] = lo[e] > 0.f ? lo[e] : palp * lo[e];
          hi[e] = hi[e] > 0.f ? hi[e] : palp * hi[e];
        }
        i32x4 o;
        o[0] = (int)((uint32_t)f32_to_bf16(lo[0]) | ((uint32_t)f32_to_bf16(lo[1]) << 16));
        o[1] = (int)((uint32_t)f32_to_bf16(lo[2]) | ((uint32_t)f32_to_bf16(lo[3]) << 16));
        o[2] = (int)((uint32_t)f32_to_bf16(hi[0]) | ((uint32_t)f32_to_bf16(hi[1]) << 16));
        o[3] = (int)((uint32_t)f32_to_bf16(hi[2]) | ((uint32_t)f32_to_bf16(hi[3]) << 16));
        asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(o) : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const SwCur lcur = ld;
    const bool llive = ld.c < cend;
    advance(ld);
    if (cp.kind != SW_COMP) {                   // halo rows only: DMA at once
#pragma unroll
      for (int i = 0; i < DMAW; ++i) issue_piece(i, LSEG, lcur, llive);
    } else {
      // 36 groups (32-pixel slice kk, tap t = 3 dy + dx); group g's reads (its B
      // fragment, plus the slice's two A fragments at t = 0) are issued PF groups
      // ahead; one DMA piece every 9 groups (a wave held up issuing a load then
      // stalls only itself)
      s16x4v ra[2][2][2], rb[PF + 1][2];        // [kk & 1][m][half], [g % (PF + 1)][half]
      uint32_t(&lbs)[3][2] = lb;
      uint32_t(&las)[2][2] = la;
      auto reads = [&](int gi) __attribute__((always_inline)) {
        const int kk = gi / 9, t = gi % 9;
        const int qk = (kk * 32) / W, x0 = (kk * 32) % W;
        if (t == 0) {
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int h = 0; h < 2; ++h) SW_TRD(ra[kk & 1][m][h], las[m][h], U * DYB + kk * 4096);
        }
        // input row y0 - 1 + qk + dy sits in ring row (U RPS - 2 + qk + dy) mod RING
        const int s = (U * RPS - 2 + qk + t / 3 + RING) % RING;
#pragma unroll
        for (int h = 0; h < 2; ++h) SW_TRD(rb[gi % (PF + 1)][h], lbs[t % 3][h], s * ROWB + x0 * 128);
      };
      auto nrd = [](int gi) { return gi >= 36 ? 0 : (gi % 9 == 0 ? 6 : 2); };
#pragma unroll
      for (int gi = 0; gi < PF; ++gi) reads(gi);
#pragma unroll
      for (int gi = 0; gi < 36; ++gi) {
        if (gi % 9 == 4 && gi / 9 < DMAW) issue_piece(gi / 9, LSEG, lcur, llive);
        if (gi + PF < 36) reads(gi + PF);
        int pend = 0;
#pragma unroll
        for (int j = 1; j <= PF; ++j) pend += nrd(gi + j);
        sw_lgkm(pend);
        const int kk = gi / 9, t = gi % 9;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          asm volatile("" : "+v"(rb[gi % (PF + 1)][h]));
#pragma unroll
          for (int m = 0; m < 2; ++m) asm volatile("" : "+v"(ra[kk & 1][m][h]));
        }
        const bf16x8 fb = __builtin_bit_cast(
            bf16x8, __builtin_shufflevector(rb[gi % (PF + 1)][0], rb[gi % (PF + 1)][1], 0, 1, 2, 3, 4, 5, 6, 7));
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const bf16x8 fa = __builtin_bit_cast(
              bf16x8, __builtin_shufflevector(ra[kk & 1][m][0], ra[kk & 1][m][1], 0, 1, 2, 3, 4, 5, 6, 7));
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[m][t], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
      }
    }
    advance(cp);
    return cp.c < cend;
  };
#pragma unroll 1
  while (true) {
    if (!step(std::integral_constant<int, 0>())) break;
    if (!step(std::integral_constant<int, 1>())) break;
    if (!step(std::integral_constant<int, 2>())) break;
    if (!step(std::integral_constant<int, 3>())) break;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- partial dW: split r of the [nwg_ps][64][9][c1 + c2] slabs reduced by
  // rr_wgrad's reduce (wgrad.hip).  Staged through LDS in two halves (m) so
  // the stores are whole 256-B rows: D rows co = 32 wc + 16 m + 4 g + e,
  // column ci = 16 wk + (lane & 15); LDS [col 32 = 16 wc + 4 g + e][tap][ci 64]
  __syncthreads();
  const int CB = a.c1 + a.c2;
  float *const pw = a.partial + ((long long)r * a.cout + ds * 64) * 9 * CB + ci0;
  float *const st = reinterpret_cast<float *>(smem);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        st[((16 * wc + 4 * g + e) * 9 + t) * 64 + 16 * wk + (lane & 15)] = acc[m][t][e];
    __syncthreads();
    for (int u = tid; u < 32 * 9 * 16; u += 512) {          // float4 units
      const int cl = u / 144, t = (u / 16) % 9, c4 = u & 15;
      const int co = (cl >> 4) * 32 + 16 * m + (cl & 15);
      *reinterpret_cast<float4 *>(pw + ((long long)co * 9 + t) * CB + c4 * 4) =
          *reinterpret_cast<const float4 *>(st + u * 4);
    }
    __syncthreads();
  }
}

}  // namespace

static int sw_slices(const rr_wgrad_desc *d) { return (d->c_in1 + d->c_in2) / 64 * (d->c_out / 64); }

int swgrad_ok(const rr_wgrad_desc *d) {
  // RR_PATH swgrad=0: the halo / tiled weight grads instead (tests)
  if (!rr_path("swgrad", 1)) return 0;
  if (d->dtype != RR_BF16 || d->mode != RR_CONV3X3 || d->c_out % 64 || d->c_out > 128) return 0;
  if (d->w != 64 && d->w != 32) return 0;
  if (d->c_in1 % 64 || d->c_in2 % 64 || d->c_in1 + d->c_in2 > 192 || d->c_in1 <= 0) return 0;
  if (d->h % (128 / d->w)) return 0;
  const long long P = (long long)d->n * d->h * d->w;
  if (P < 128LL * SW_WG || P * 192 > INT_MAX) return 0;
  return 1;
}

int swgrad_nsplit(const rr_wgrad_desc *d) { return SW_WG / sw_slices(d); }

int swgrad_launch(const rr_wgrad_desc *d, const void *dy, const void *x1, const void *x2, void *ws,
                  hipStream_t st) {
  const int S = sw_slices(d);
  SWArgs a;
  a.dy = (const char *)dy;
  a.x1 = (const char *)x1;
  a.x2 = (const char *)x2;
  a.c1 = d->c_in1;
  a.c2 = d->c_in2;
  a.cout = d->c_out;
  a.partial = (float *)ws;
  a.n = d->n;
  a.h = d->h;
  a.nwg_ps = SW_WG / S;
  a.nsteps = (int)((long long)d->n * d->h * d->w / 128);
  const dim3 grid(a.nwg_ps * S), block(512);
  a.pre_s = a.pre_b = a.pre_alpha = nullptr;
  if (d->w == 64) hipLaunchKernelGGL((swgrad_kernel<64, false>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((swgrad_kernel<32, false>), grid, block, 0, st, a);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

int swgrad_launch_pre(const rr_wgrad_desc *d, const void *dy, const void *x1, const float *pre_s,
                      const float *pre_b, const float *pre_alpha, void *ws, hipStream_t st) {
  if (!swgrad_ok(d) || d->c_in2 || !pre_s || !pre_b || !pre_alpha) return RR_EUNSUPPORTED;
  const int S = sw_slices(d);
  SWArgs a;
  a.dy = (const char *)dy;
  a.x1 = (const char *)x1;
  a.x2 = nullptr;
  a.c1 = d->c_in1;
  a.c2 = 0;
  a.cout = d->c_out;
  a.partial = (float *)ws;
  a.n = d->n;
  a.h = d->h;
  a.nwg_ps = SW_WG / S;
  a.nsteps = (int)((long long)d->n * d->h * d->w / 128);
  a.pre_s = pre_s; a.pre_b = pre_b; a.pre_alpha = pre_alpha;
  const dim3 grid(a.nwg_ps * S), block(512);
  if (d->w == 64) hipLaunchKernelGGL((swgrad_kernel<64, true>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((swgrad_kernel<32, true>), grid, block, 0, st, a);
  RR_CHECK_LAUNCH();
  return RR_OK;
}
