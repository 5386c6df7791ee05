// stream3.hip -- row-streaming 3x3 bf16 convolution for the wide, shallow
// layers (64 -> 64 channels on 64x64 and 32x32 maps): res1 / dec1 / dec2
// conv fwd + dgrad + the fused BN/PReLU-backward dgrad of ResUNet
// (14_train_unified_advanced.py:96-115) and the VGG16 conv1_2 of the
// perceptual loss (14:189-196).
//
// Why a separate kernel.  At 64 channels a 3x3 conv is HBM-bound on MI355X
// (K = 576: ~270 FLOP per byte moved, under the MFMA/HBM ridge), so what
// matters is streaming the activations once at full bandwidth.  The tiled
// halo kernel (igemm.hip) re-reads 1.5x of the input per tile, re-reads the
// weights from L2 for every tile and only overlaps a tile's loads with the
// other workgroup's MFMAs.  Here:
//   * one persistent 512-thread workgroup per CU walks a contiguous range of
//     output rows (whole images at batch 512) in steps of SPX = 64 MP
//     pixels (RPS = SPX / W image rows);
//   * every input row is read ONCE: rows land by LDS-DMA
//     (global_load_lds_dwordx4) in a ring of RING padded rows, D steps ahead
//     of the MFMAs; a step's three input-row windows for the taps are slots
//     of that ring (the zero padding rows / columns come from a zero page);
//   * the weights (64 x 576 bf16 = 72 KB) live in registers for the whole
//     kernel: wave (wc, wp) owns output channels [32 wc, 32 wc + 32) -- its
//     A fragments, 144 VGPRs -- and 16 MP pixels of each step;
//   * the epilogue (compile-time flags F) stores from the accumulators (4
//     NHWC channels per lane) and keeps BN statistics / BN-backward sums in
//     registers across all the workgroup's steps (one reduction at the end,
//     per-workgroup partials).
// The per-step scalar work (ring slots, DMA addresses, cursor, waits) is
// fixed, so epilogues without global loads use 256-pixel steps (MP = 4),
// twice the MFMA work per unit of overhead; those with loads (accumulate,
// relu mask, BN backward) keep 128-pixel steps for their operand registers.
//
// Ring row image: the W + 2 zero-padded pixels of an input row, 128 B each
// (64 channels), pixel-major, with the 16-B channel chunks of pixel p
// XOR-permuted: slot s of pixel p holds chunk s ^ swz(p mod 16).  A DMA
// piece is then 8 whole pixels = 1 KB of contiguous NHWC input (8 cache
// lines per instruction instead of 64 for a channel-planar image), and the
// MFMA B reads stay conflict-free: a ds_read_b128 16-lane group reads 16
// consecutive pixels, 8 at chunk c and 8 at chunk c + 1 (c even); swz (see
// s3_swz) makes those 16 bank slots distinct for pixel offsets 0, 1, 2 mod
// 16 -- the three tap columns of a 16-pixel block, the only offsets read.
//
// vmcnt accounting: LDS-DMA, the epilogue's global loads and its stores share
// the in-order vector-memory counter.  Iteration u issues, in this order:
// epilogue loads E(u), DMA(u + D) (DMAW per wave), stores S(u).  Before step
// v reads the ring, a wave waits until at most
//   (D - 1) DMAW + S [v-D computed] + (E + S) * #computed in (v-D, v)
// of its ops are outstanding (exactly the ops younger than DMA(v)), then a
// raw s_barrier publishes every wave's rows.  A plain __syncthreads would
// drain all DMA in flight (vmcnt(0)).  The epilogue loads and the B-fragment
// reads are inline asm with their own counted waits: with an LDS-DMA in
// flight hipcc waits vmcnt(0) / lgkmcnt(0) for the results of ordinary
// loads, which would drain the prefetch every step.
#include "common.h"
#include "stream3.h"

#include <climits>
#include <cstdlib>
#include <type_traits>

// B fragments of the three tap columns: 3 reads per (tap row, k half).
// Forming the dx = 0 / 2 operands by DPP row rotates of one centre read (a
// third of the LDS fragment traffic) measured 15 % slower on the stream3
// layers and -1.1 % on the graph step (profiles/r5n_ablayers_s3.txt,
// r5n_ablibs.txt): the LDS port was not the limiter.

#ifdef RR_S3_STAMPS
// diagnostic build only (make s3stamps; tools/s3_stamps.py): per-wave sums of
// the step loop's segments, read with rr_s3_stamps; never shipped
__device__ unsigned long long rr_s3_stamps[256 * 8 * 8];
#define S3_STAMP(t)                                                             \
  do {                                                                          \
    __builtin_amdgcn_sched_barrier(0);                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");   \
    __builtin_amdgcn_sched_barrier(0);                                          \
  } while (0)
#else
#define S3_STAMP(t) do {} while (0)
#endif

namespace {

constexpr int S3_WG = 256;   // workgroups: one per CU on MI355X (fixed: deterministic partial rows)

// F_POOL: the 2x2 max-pool (+ its first-max index) of the activated output
// instead of the output (VGG16 conv + ReLU + MaxPool2d, 14:189-196)
// F_SC: a 1x1 dgrad of a second gradient (a.xsc, weights a.wsc) summed into
// the accumulators -- the shortcut conv's dgrad of a ResidualBlock with a
// concat input, 14:109-113 (rr_igemm_dgrad_sc)
// F_PRELU / F_RES: the BN-folded eval forward's epilogues (rr_igemm_ex,
// 17:84-86 through 14:96-115): PReLU(conv + b) of conv1, act(conv + b + x)
// of an identity-shortcut conv2 (the residual added after the bias, as the
// tap-reuse conv's register epilogue); F_PFULL: with F_POOL, the full-size
// output is stored too (an encoder block's skip tensor); F_PNOIDX: with
// F_POOL, no window index (nothing runs backward)
enum : int { F_BIAS = 1, F_STATS = 2, F_RELU = 4, F_ACC = 8, F_MASK = 16, F_BNBWD = 32, F_POOL = 64,
             F_SC = 128, F_PRELU = 256, F_RES = 512, F_PFULL = 1024, F_PNOIDX = 2048, F_PRE = 4096 };
// F_PRE: the input is the pre-BN t1 of a ResidualBlock's conv1; every row
// that lands in the ring is turned into a1 = PReLU(t1 * s + b) in LDS (the
// bytes rr_affine_act would have written: the same fp32 expression and bf16
// rounding) before any step reads it -- BN1 + PReLU folded into conv2's
// forward (14:101-104), the a1 tensor never stored

// chunk swizzle: the 16 pixels of a B read at pixel offset P in {0, 1, 2}
// mod 16 need distinct (p & 1, chunk ^ swz(p)) pairs with chunks c (outer 8
// lanes) and c + 1 (inner 8); for each pixel parity the 8 values e_k =
// swz(2k + parity) must satisfy {e0,e1,e2^1,e3^1,e4^1,e5^1,e6,e7} and
// {e0,e1,e2,e3^1,e4^1,e5^1,e6^1,e7} both = {0..7}, i.e. e2 == e6 and the
// other six fill the rest: e = 2 3 0 5 4 7 0 7 (checked for every lane group)
__host__ __device__ constexpr int s3_swz(int p) { return (0x70745032u >> (4 * ((p >> 1) & 7))) & 0xf; }

template <int W, int MP> struct S3Geo {
  static constexpr int SPX = 64 * MP;                          // pixels per step
  static constexpr int RPS = SPX / W;                          // image rows per step
  // padded pixels per ring row: >= W + 2, and a step's rows split into whole
  // 1-KB DMA pieces over the 8 waves
  static constexpr int RPX = W == 32 ? 48 : (MP == 4 ? 80 : 96);
  static constexpr int ROWB = RPX * 128;                       // one padded row, 64 channels
  static constexpr int SCRATCH = 2048;                         // bnbwd coefficients
  static constexpr int RING = (160 * 1024 - SCRATCH) / ROWB;   // ring rows
  static constexpr int D = (RING - 2) / RPS - 1;               // steps of prefetch in flight
  static constexpr int DMAW = RPS * ROWB / 8192;               // DMA instructions / wave / step
  static constexpr int LDS = RING * ROWB + SCRATCH;
  static_assert((RPS * ROWB) % 8192 == 0, "a step's rows must split evenly over 8 waves");
  static_assert(ROWB % 1024 == 0, "DMA pieces never straddle ring rows");
  static_assert(RPX >= W + 2 && ROWB % 256 == 0, "row size");
  static_assert(D >= 2 && (D + 1) * RPS + 2 <= RING, "ring");
  static_assert(LDS <= 160 * 1024, "LDS");
};

enum { S3_PRE = 0, S3_COMP = 1 };

#define S3_W1(n) \
  case n: asm volatile("s_waitcnt vmcnt(" #n ")\n\ts_barrier" ::: "memory"); break;
#define S3_W8(b) S3_W1(b) S3_W1(b + 1) S3_W1(b + 2) S3_W1(b + 3) S3_W1(b + 4) S3_W1(b + 5) \
  S3_W1(b + 6) S3_W1(b + 7)

// wait until at most n of this wave's vector-memory ops are outstanding, then
// a workgroup barrier (n is wave-uniform; s_waitcnt needs an immediate)
__device__ __forceinline__ void wait_vm_barrier(int n) {
  switch (n < 0 ? 0 : (n > 63 ? 63 : n)) {
    S3_W8(0) S3_W8(8) S3_W8(16) S3_W8(24) S3_W8(32) S3_W8(40) S3_W8(48) S3_W8(56)
    default: asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory"); break;
  }
}
template <int N> __device__ __forceinline__ void wait_vm_barrier_c() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

typedef unsigned long long u64;
typedef int i32x4 __attribute__((ext_vector_type(4)));

// 8-byte global load the compiler's waitcnt pass does not see (the caller
// waits with an explicit vmcnt that names the result registers)
__device__ __forceinline__ u64 load_b64_async(const char *p) {
  u64 r;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
// (16 B: a B fragment of the F_SC source)
__device__ __forceinline__ i32x4 load_b128_async(const char *p) {
  i32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
// LDS reads outside the compiler's view: its waitcnt pass puts a vmcnt(0)
// (drain all LDS-DMA) before a visible ds_read it cannot separate from the
// DMA destination
__device__ __forceinline__ f32x4 lds_read_4(const float *p) {
  f32x4 r;
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
  return r;
}
// (early-clobber outputs: the first read's destination must not be the
// second read's address register -- the LDS queue can hold the second read
// past the first one's data return)
__device__ __forceinline__ void lds_read_2x4(const float *p, f32x4 &lo, f32x4 &hi) {
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(lo), "=&v"(hi) : "v"(a) : "memory");
}
__device__ __forceinline__ f32x4 unpack4(u64 v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  return f32x4{__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
               __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
}
__device__ __forceinline__ uint2 pack4(f32x4 g) {
  uint2 o;
  o.x = (uint32_t)f32_to_bf16(g[0]) | ((uint32_t)f32_to_bf16(g[1]) << 16);
  o.y = (uint32_t)f32_to_bf16(g[2]) | ((uint32_t)f32_to_bf16(g[3]) << 16);
  return o;
}

template <int N> using ic = std::integral_constant<int, N>;

// a wave's MP 16-pixel blocks of a step: block ni sits brow(ni) image rows and
// bcol(ni) columns from the wave's first pixel (POOL: 2 rows x 8 MP columns,
// blocks 2j / 2j + 1 = rows 0 / 1 of columns 16 j ..)
template <int W, int MP, bool POOL> struct S3Blk {
  static constexpr int brow(int ni) { return POOL ? (ni & 1) : (ni * 16) / W; }
  static constexpr int bcol(int ni) { return POOL ? (ni >> 1) * 16 : (ni * 16) % W; }
};

// virtual step: pre-load, or compute of output rows [y0, y0 + RPS) of the
// column (image img, columns [xs, xs + W)); a column is a whole image on the
// 32 / 64-wide maps, a W-wide strip of it on the wider ones (column-strip
// mode: the strip's left / right neighbour pixels are its halo)
struct Cur {
  int kind, img, xs, y0, c;
};

// SM: column-strip mode (a.w a multiple of W); whole rows (a.w == W) keep
// the width a compile-time constant
template <int W, int MP, int F, int STAG, bool SM>
__global__ __launch_bounds__(512, 2) void stream3_kernel(S3Args a, int nsteps) {
  using G = S3Geo<W, MP>;
  constexpr int RPS = G::RPS, ROWB = G::ROWB, RING = G::RING, D = G::D;
  constexpr int DMAW = G::DMAW;
  constexpr int MC = 2;                         // 32 output channels per wave
  constexpr bool BNBWD = (F & F_BNBWD) != 0;
  constexpr bool ACC = (F & F_ACC) != 0, MASK = (F & F_MASK) != 0;
  constexpr bool STATS = (F & F_STATS) != 0;
  constexpr bool POOL = (F & F_POOL) != 0;
  constexpr bool SC = (F & F_SC) != 0;
  constexpr bool RES = (F & F_RES) != 0, PRELU = (F & F_PRELU) != 0;
  constexpr bool PFULL = (F & F_PFULL) != 0, PIDX = POOL && !(F & F_PNOIDX);
  constexpr bool PRE = (F & F_PRE) != 0;
  static_assert(!PRE || (F == (F_BIAS | F_STATS | F_PRE) && STAG == 0 && !SM), "input transform: the BN-statistics forward");
  static_assert(!SC || (F == F_SC && STAG == 0), "the 1x1 second source: plain dgrad epilogue");
  static_assert(!POOL || ((F & ~(F_BIAS | F_RELU | F_POOL | F_RES | F_PFULL | F_PNOIDX)) == 0 && (F & F_RELU) &&
                          MP % 2 == 0 && W % (8 * MP) == 0), "pool epilogue: bias + ReLU, row-pair blocks");
  static_assert(!(RES && (ACC || BNBWD || STATS)) && !(PRELU && (F & F_RELU)), "epilogue flag set");
  constexpr int NE = BNBWD ? 1 : (ACC ? 1 : 0) + (MASK ? 1 : 0) + (RES ? 1 : 0);   // epilogue loads per block
  // S: stores per step (16-B output stores; POOL: a pooled value (+ an index)
  // store per channel block and column block pair, + the full output's)
  // (F_SC: its B fragments, 2 k-halves per pixel block, count with the
  // epilogue loads: issued with them, waited for after the 3x3 MFMAs)
  constexpr int E = MC * MP * NE + (SC ? 2 * MP : 0);
  constexpr int S = POOL ? (MC * MP / 2) * (PIDX ? 2 : 1) + (PFULL ? MP : 0) : MP;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  float *coef = reinterpret_cast<float *>(smem + RING * ROWB);   // [64][2]

  const int tid = threadIdx.x, lane = tid & 63;
  // wave-uniform indices in SGPRs (the address math of a step is scalar)
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wv & 1, wp = wv >> 1;
  const int frow = lane & 15, fq = lane >> 4;
  const int H = a.h;
  const int IW = SM ? a.w : W;                  // image width: W (whole rows) or a multiple of it (strips)
  const int spi = H / RPS;                      // compute steps per column
  const int cbeg = (int)((long long)blockIdx.x * nsteps / S3_WG);
  const int cend = (int)((long long)(blockIdx.x + 1) * nsteps / S3_WG);

  // ---- weights -> registers: A fragments of channels wc*32 + mi*16 + frow ----
  bf16x8 wr[MC][9][2];
#pragma unroll
  for (int mi = 0; mi < MC; ++mi) {
    const int co = wc * 32 + mi * 16 + frow;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        wr[mi][tap][kb] =
            *reinterpret_cast<const bf16x8 *>(a.wt + ((co * 9 + tap) * a.wld + a.woff + kb * 32 + fq * 8) * 2);
  }
  // F_SC: the 1x1 weights [c_out][64] of the wave's output channels
  bf16x8 wsr[SC ? MC : 1][2];
  if constexpr (SC) {
#pragma unroll
    for (int mi = 0; mi < MC; ++mi) {
      const int co = wc * 32 + mi * 16 + frow;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        wsr[mi][kb] = *reinterpret_cast<const bf16x8 *>(a.wsc + (co * 64 + kb * 32 + fq * 8) * 2);
    }
  }
  float al = 0.f;
  if constexpr (BNBWD) {
    if (tid < 64) {
      // u = t * s + b (BN out = PReLU in)
      coef[tid * 2 + 0] = a.baff_s[tid];
      coef[tid * 2 + 1] = a.baff_b[tid];
    }
    al = a.balpha[0];
    __syncthreads();
  }
  // BNBWD: the wave's (s, b) coefficients in registers for the whole loop
  // (two LDS round trips with a full lgkmcnt wait per step otherwise)
  f32x4 bk[BNBWD ? MC : 1][2];
  if constexpr (BNBWD) {
#pragma unroll
    for (int mi = 0; mi < MC; ++mi) lds_read_2x4(coef + (wc * 32 + mi * 16 + fq * 4) * 2, bk[mi][0], bk[mi][1]);
  }
  // the bias in registers for the whole loop (read from the LDS per step,
  // behind a full lgkmcnt wait, until round 6)
  f32x4 biar[(F & F_BIAS) ? MC : 1];
  const float alp = PRELU ? a.alpha[0] : 0.f;   // (resident with the weights: the vmcnt(0) below)
  // F_PRE: a thread transforms chunks tid + 512 j of a step's new rows, all
  // at the same ring-row pixel and 16-B slot (512 is a multiple of a row's
  // W x 8 slots): its 8 channels' (s, b) in registers
  f32x4 pcs[PRE ? 2 : 1], pcb[PRE ? 2 : 1];
  float palp = 0.f;
  if constexpr (PRE) {
    const int rem = tid % (W * 8);
    const int px = 1 + (rem >> 3), c = (rem & 7) ^ s3_swz(px & 15);
    pcs[0] = *reinterpret_cast<const f32x4 *>(a.pre_s + 8 * c);
    pcs[1] = *reinterpret_cast<const f32x4 *>(a.pre_s + 8 * c + 4);
    pcb[0] = *reinterpret_cast<const f32x4 *>(a.pre_b + 8 * c);
    pcb[1] = *reinterpret_cast<const f32x4 *>(a.pre_b + 8 * c + 4);
    palp = a.pre_alpha[0];
  }
  if constexpr ((F & F_BIAS) != 0) {
    if (tid < 64) coef[tid] = a.bias[tid];
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < MC; ++mi) biar[mi] = lds_read_4(coef + wc * 32 + mi * 16 + fq * 4);
  }

  // ---- LDS-DMA pieces: a 1-KB piece lies in one ring row, so its row and
  // chunk are wave-uniform; the lane's plane / pixel is fixed.  A wave's
  // DMAW consecutive pieces lie in ONE ring row (a row is a whole multiple of
  // them), so the row's terms (image row, validity, source base, ring slot)
  // are formed once per step, and the lane's padding select is arithmetic:
  // the scalar unit, shared by the CU's 8 waves, and an exec-mask region per
  // piece had made the DMA issue ~16 % of a step (profiles/r6h_s3_stamps.jsonl) ----
  static_assert((ROWB / 1024) % DMAW == 0, "a wave's pieces share one ring row");
  const long long zoff = (long long)((uintptr_t)rr_zero_page - (uintptr_t)a.x);   // zero source
  const int drow = (wv * DMAW * 1024) / ROWB;       // the wave's ring row within a step (uniform)
  static_assert(DMAW <= 8, "piece bits");
  int dchk[DMAW];
  int dofs[DMAW];                                   // lane source offset from the column's pixel 0
  // lane pixel of piece i: bit i inside the column, bit 8 + i its left
  // neighbour, bit 16 + i its right one (one register for all pieces)
  uint32_t dcode = 0;
#pragma unroll
  for (int i = 0; i < DMAW; ++i) {
    const int piece = (wv * DMAW + i) * 1024;
    dchk[i] = piece - drow * ROWB;
    const int o = dchk[i] + lane * 16;
    const int px = o / 128, x = px - 1, chunk = ((o / 16) & 7) ^ s3_swz(px & 15);
    dofs[i] = x * 128 + chunk * 16;
    dcode |= (x >= 0 && x < W ? 1u : 0u) << i;
    dcode |= (x == -1 ? 1u : 0u) << (8 + i);
    dcode |= (x == W ? 1u : 0u) << (16 + i);
  }
  // DMA of virtual step `cu` into the ring rows starting at slot `slot`
  auto issue = [&](int slot, const Cur &cu, bool live) __attribute__((always_inline)) {
    const int y = cu.kind == S3_PRE ? cu.y0 - RPS + 1 + drow : cu.y0 + 1 + drow;
    const bool rok = live & (y >= 0) & (y < H) & ((cu.kind != S3_PRE) | (drow >= RPS - 2));   // uniform
    // the column's neighbour pixels are real ones inside the image (strips)
    const bool lm = SM && cu.xs > 0, rm = SM && cu.xs + W < IW;                              // uniform
    const uint32_t okb = (dcode | (lm ? dcode >> 8 : 0u) | (rm ? dcode >> 16 : 0u)) & 0xffu;
    // (an invalid row reads the zero page: its base makes every lane's
    // candidate land there)
    const long long rbase = rok ? ((long long)(cu.img * H + y) * IW + cu.xs) * 128 : zoff;
    int s = slot + drow;
    s = s >= RING ? s - RING : s;
    char *const dst = smem + s * ROWB;
#pragma unroll
    for (int i = 0; i < DMAW; ++i) {
      // one base pointer + a selected offset (no pointer select / branch:
      // two exec-masked DMA instructions would break the vmcnt accounting)
      const long long m = ((okb >> i) & 1u) ? 0LL : -1LL;   // -1: padding lane
      const long long cand = rok ? rbase + dofs[i] : zoff;
      const long long off = (cand & ~m) | (zoff & m);
      __builtin_amdgcn_global_load_lds((const void *)(a.x + off), LDS_PTR(dst + dchk[i]), 16, 0, 0);
    }
  };
  auto advance = [&](Cur &cu) __attribute__((always_inline)) {
    if (cu.kind == S3_PRE) {
      cu.kind = S3_COMP;
    } else {
      ++cu.c;
      cu.y0 += RPS;
      if (cu.y0 == H) {
        cu.y0 = 0;
        cu.xs += W;
        if (cu.xs == IW) { cu.xs = 0; ++cu.img; }
        cu.kind = S3_PRE;
      }
    }
  };

  // ---- per-wave pixel blocks of a step and lane parts ----
  // the wave's 16 MP pixels start at row q0, column x0 (uniform); block ni
  // sits brow(ni) rows and bcol(ni) columns further (compile time: x0 + 16 MP
  // never crosses more than the rows the geometry implies).  POOL: a wave
  // owns 2 rows x 8 MP columns (blocks 2j / 2j + 1 = rows 0 / 1 of columns
  // 16 j ..), so a 2x2 window lies in one lane and its xor-1 neighbour
  constexpr int NR = POOL ? 2 : (16 * MP + W - 1) / W;   // distinct image rows of a wave's pixels
  constexpr int PCOLS = 8 * MP, WPR = POOL ? W / PCOLS : 1;
  const int q0 = POOL ? 2 * (wp / WPR) : (wp * 16 * MP) / W;
  const int x0 = POOL ? PCOLS * (wp % WPR) : (wp * 16 * MP) % W;
  static_assert(W >= 16 * MP || (16 * MP) % W == 0, "block rows");
  using BK = S3Blk<W, MP, POOL>;
  auto brow = [](int ni) constexpr { return BK::brow(ni); };
  auto bcol = [](int ni) constexpr { return BK::bcol(ni); };
  // lane part of a B read for tap column dx and k-half kb: pixel frow + dx of
  // the block, chunk kb * 4 + fq through the swizzle
  uint32_t boff[3][2];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
      boff[dx][kb] = (frow + dx) * 128 + (((kb * 4 + fq) ^ s3_swz((frow + dx) & 15)) * 16);
  const uint32_t sbase = (uint32_t)(uintptr_t)smem;
  const uint32_t le = (frow * 64 + wc * 32 + fq * 4) * 2;                // lane part of an output (acc layout)
  // widened stores (permlane16 swaps, see epilogue): lane part of a 16-B store
  const uint32_t le2 = frow * 128 + (wc * 32 + (fq & 1) * 16 + (fq & 2) * 4) * 2;

  // running epilogue sums: stats (sum, sum sq) or bnbwd (sum gm, sum gm t)
  f32x4 r0[MC], r1[MC];
  float ra = 0.f;
#pragma unroll
  for (int mi = 0; mi < MC; ++mi) { r0[mi] = f32x4{0.f, 0.f, 0.f, 0.f}; r1[mi] = r0[mi]; }

  u64 ev0[MC][MP], ev1[MC][MP];
  i32x4 esc[SC ? MP : 1][2];                    // F_SC B fragments: pixel frow, channels kb * 32 + fq * 8
  f32x4 acc[MC][MP];
  auto load_e = [&](long long pix0) __attribute__((always_inline)) {
    if constexpr (SC) {
#pragma unroll
      for (int ni = 0; ni < MP; ++ni) {
        const long long ub = (pix0 + (q0 + brow(ni)) * IW + x0 + bcol(ni)) * 128;   // uniform
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) esc[ni][kb] = load_b128_async(a.xsc + ub + frow * 128 + kb * 64 + fq * 16);
      }
    }
#pragma unroll
    for (int mi = 0; mi < MC; ++mi)
#pragma unroll
      for (int ni = 0; ni < MP; ++ni) {
        const long long ub = (pix0 + (q0 + brow(ni)) * IW + x0 + bcol(ni)) * 128 + mi * 32;   // uniform
        if constexpr (BNBWD) ev0[mi][ni] = load_b64_async(a.bt + ub + le);
        if constexpr (!BNBWD && ACC) ev0[mi][ni] = load_b64_async(a.y + ub + le);
        if constexpr (RES) ev0[mi][ni] = load_b64_async(a.res + ub + le);
        if constexpr (!BNBWD && MASK) ev1[mi][ni] = load_b64_async(a.mask + ub + le);
      }
  };
  auto wait_e = [&]() __attribute__((always_inline)) {
    // the epilogue loads are older than the DMAW DMAs issued after them
    if constexpr (E > 0) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMAW) : "memory");
      if constexpr (SC) {
#pragma unroll
        for (int ni = 0; ni < MP; ++ni)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) asm volatile("" : "+v"(esc[ni][kb]));
      }
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int ni = 0; ni < MP; ++ni) {
          if constexpr (BNBWD || ACC || RES) asm volatile("" : "+v"(ev0[mi][ni]));
          if constexpr (MASK && !BNBWD) asm volatile("" : "+v"(ev1[mi][ni]));
        }
    }
  };
  auto mfma_step = [&](int s0) __attribute__((always_inline)) {
    // ring slot of input row y0 - 1 + r is s0 + r (mod RING); s0 + r < 2 RING
    uint32_t rba[3][NR];                        // per tap row dy and image row: ring row base (uniform)
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        int r = s0 + q0 + k + dy;
        r = r >= RING ? r - RING : r;
        rba[dy][k] = sbase + r * ROWB + x0 * 128;
      }
    // 18 (tap, k-half) groups; the B fragments of group q + 1 are read before
    // group q's MFMAs (counted lgkmcnt(MP): the prefetched group stays in flight)
    i32x4 fb[2][MP];
#pragma unroll
    for (int ni = 0; ni < MP; ++ni)
      asm volatile("ds_read_b128 %0, %1 offset:%2"
                   : "=v"(fb[0][ni]) : "v"(rba[0][brow(ni)] + boff[0][0]),
                     "i"(bcol(ni) * 128));
#pragma unroll
    for (int q = 0; q < 18; ++q) {
      if (q + 1 < 18) {
        const int t1 = (q + 1) >> 1, kb1 = (q + 1) & 1;
#pragma unroll
        for (int ni = 0; ni < MP; ++ni)
          asm volatile("ds_read_b128 %0, %1 offset:%2"
                       : "=v"(fb[(q + 1) & 1][ni])
                       : "v"(rba[t1 / 3][brow(ni)] + boff[t1 % 3][kb1]),
                         "i"(bcol(ni) * 128));
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(MP) : "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
#pragma unroll
      for (int ni = 0; ni < MP; ++ni) asm volatile("" : "+v"(fb[q & 1][ni]));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int ni = 0; ni < MP; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              wr[mi][q >> 1][q & 1], __builtin_bit_cast(bf16x8, fb[q & 1][ni]),
              q == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mi][ni], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  // epilogue: lane = pixel (frow) x 4 channels of each 16 x 16 block
  // (pix0: the step's first output pixel, rowg: its image row over the batch,
  // xs: the column's first image column)
  auto epilogue = [&](long long pix0, int rowg, int xs) __attribute__((always_inline)) {
    uint2 pk[MC][MP];
#pragma unroll
    for (int mi = 0; mi < MC; ++mi) {
      f32x4 k01, k23;                           // (s, b) of the lane's 4 channels
      if constexpr (BNBWD) { k01 = bk[mi][0]; k23 = bk[mi][1]; }
      f32x4 bia;
      if constexpr ((F & F_BIAS) != 0) bia = biar[mi];
#pragma unroll
      for (int ni = 0; ni < MP; ++ni) {
        f32x4 g = acc[mi][ni];
        if constexpr (BNBWD) {
          const f32x4 t = unpack4(ev0[mi][ni]);
          f32x4 gm;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            // sum gm * xhat = inv (sum gm t) - inv mean (sum gm): the affine
            // part is applied once per channel at the end
            const float ks = j < 2 ? k01[2 * j] : k23[2 * j - 4];
            const float kb = j < 2 ? k01[2 * j + 1] : k23[2 * j - 3];
            const float u = t[j] * ks + kb;
            ra += u > 0.f ? 0.f : g[j] * u;
            gm[j] = u > 0.f ? g[j] : al * g[j];
            r0[mi][j] += gm[j];
            r1[mi][j] += gm[j] * t[j];
          }
          g = gm;
        } else {
          // ACC: the destination holds the first pass of a two-source (concat)
          // conv, so the statistics and the bias apply to the sum
          if constexpr (ACC) g += unpack4(ev0[mi][ni]);
          if constexpr (STATS) {
            r0[mi] += g;
            r1[mi] += g * g;
          }
          if constexpr ((F & F_BIAS) != 0) g += bia;
          if constexpr (RES) g += unpack4(ev0[mi][ni]);
          if constexpr ((F & F_RELU) != 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) g[j] = fmaxf(g[j], 0.f);
          }
          if constexpr (PRELU) {
#pragma unroll
            for (int j = 0; j < 4; ++j) g[j] = g[j] > 0.f ? g[j] : alp * g[j];
          }
          if constexpr (MASK) {
            const f32x4 mk = unpack4(ev1[mi][ni]);
#pragma unroll
            for (int j = 0; j < 4; ++j) g[j] = mk[j] > 0.f ? g[j] : 0.f;
          }
        }
        pk[mi][ni] = pack4(g);
      }
    }
    if constexpr (POOL) {
      // the 2x2 window (rows q0, q0 + 1 of columns x0 + 16 j + frow and its
      // xor-1 neighbour lane) on the bf16-rounded values -- the stored ones
      // maxpool_fwd8 would read -- in window order, first max + its index
      const long long prow = (rowg + q0) >> 1;                    // pooled row (uniform)
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int j = 0; j < MP / 2; ++j) {
          const uint2 a0 = pk[mi][2 * j], a1 = pk[mi][2 * j + 1];
          const uint2 b0 = make_uint2(xor1_u32(a0.x), xor1_u32(a0.y));
          const uint2 b1 = make_uint2(xor1_u32(a1.x), xor1_u32(a1.y));
          const f32x4 u0 = unpack4(((u64)a0.y << 32) | a0.x), v0 = unpack4(((u64)b0.y << 32) | b0.x);
          const f32x4 u1 = unpack4(((u64)a1.y << 32) | a1.x), v1 = unpack4(((u64)b1.y << 32) | b1.x);
          f32x4 m;
          uint32_t id[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) m[c] = pool4_first_max(u0[c], v0[c], u1[c], v1[c], id[c]);
          if ((frow & 1) == 0) {
            const long long pp = prow * (IW / 2) + ((xs + x0 + 16 * j + frow) >> 1);
            const int c = wc * 32 + mi * 16 + fq * 4;
            *reinterpret_cast<uint2 *>(a.ypool + (pp * 64 + c) * 2) = pack4(m);
            if constexpr (PIDX)
              *reinterpret_cast<uint32_t *>(a.pidx + pp * 64 + c) = id[0] | (id[1] << 8) | (id[2] << 16) | (id[3] << 24);
          }
        }
      if constexpr (!PFULL) return;
    }
    // widened stores: per pixel-block pair (A, B) two permlane16 swap levels
    // turn the accumulator layout (lane: 4 channels of one pixel) into 16 B
    // per lane, 4 lanes = the wave's 32 channels (64 B) of one pixel:
    //  1. per mi, swap(A, B) on each dword: rows 0/2 hold 8 channels of A's
    //     pixel, rows 1/3 8 channels of B's (odd rows of vdst <-> even rows
    //     of src);
    //  2. swap(mi 0, mi 1) on each of the 4 dwords: register 0 holds pixel A,
    //     register 1 pixel B, channel start (fq & 1) * 16 + (fq & 2) * 4.
    // 16 swaps + MP/2 * 2 16-B stores instead of 2 MP 8-B stores.
#pragma unroll
    for (int j = 0; j < MP / 2; ++j) {
      uint32_t v[MC][4];
#pragma unroll
      for (int mi = 0; mi < MC; ++mi) {
        const auto rx = __builtin_amdgcn_permlane16_swap(pk[mi][2 * j].x, pk[mi][2 * j + 1].x, false, false);
        const auto ry = __builtin_amdgcn_permlane16_swap(pk[mi][2 * j].y, pk[mi][2 * j + 1].y, false, false);
        v[mi][0] = rx[0]; v[mi][1] = ry[0]; v[mi][2] = rx[1]; v[mi][3] = ry[1];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const auto r = __builtin_amdgcn_permlane16_swap(v[0][k], v[1][k], false, false);
        v[0][k] = r[0];
        v[1][k] = r[1];
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ni = 2 * j + h;
        const long long ub = (pix0 + (q0 + brow(ni)) * IW + x0 + bcol(ni)) * 128;   // uniform
        *reinterpret_cast<uint4 *>(a.y + ub + le2) = make_uint4(v[h][0], v[h][1], v[h][2], v[h][3]);
      }
    }
  };

  // weights / bias / coefficients resident before any DMA is in flight: the
  // compiler's own wait for them would otherwise drain the prologue DMAs
  __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0) (gfx9 encoding)
  Cur ld;
  {
    const int col = cbeg / spi, ns = IW / W;    // column, columns per image
    ld.c = cbeg;
    ld.img = col / ns;
    ld.xs = (col - ld.img * ns) * W;
    ld.y0 = (cbeg - col * spi) * RPS;
    ld.kind = S3_PRE;
  }
  Cur cp = ld;
  int lslot = 0;                                // ring slot of the loader's step
#pragma unroll
  for (int k = 0; k < D; ++k) {
    issue(lslot, ld, ld.c < cend);
    advance(ld);
    lslot += RPS;
    lslot = lslot >= RING ? lslot - RING : lslot;
  }
  int cslot = RING - 2;                         // ring slot of the compute step's row y0 - 1
  // F_PRE: BN1 + PReLU of the rows DMA'd for virtual step c (ring slots cs +
  // 2 + r: a compute step's image rows y0 + 1 + r, a pre-load's y0 - 1 and
  // y0).  Done one step ahead -- step v + 1's rows at the end of iteration v,
  // whose barrier waited for DMA(v + 1) instead of DMA(v) -- so the next
  // iteration's barrier publishes them: no barrier of its own, and the work
  // overlaps the other waves' MFMAs (no step reads them before: step v's rows
  // are y0 - 1 .. y0 + RPS)
  auto pre_rows = [&](const Cur &c, int cs) __attribute__((always_inline)) {
    if constexpr (PRE) {
      const bool cmp = c.kind == S3_COMP;
      constexpr int NCH = RPS * W * 8;
      static_assert(NCH % 512 == 0, "whole chunks per thread");
#pragma unroll
      for (int j = 0; j < NCH / 512; ++j) {
        const int k = tid + 512 * j;
        const int r = k / (W * 8), rem = k - r * (W * 8);
        const int px = 1 + (rem >> 3);
        const int y = cmp ? c.y0 + 1 + r : c.y0 - RPS + 1 + r;
        if (y < 0 || y >= H || (!cmp && r < RPS - 2)) continue;
        int sl = cs + 2 + r;
        sl = sl >= RING ? sl - RING : sl;
        const uint32_t addr = sbase + sl * ROWB + px * 128 + (rem & 7) * 16;
        i32x4 v;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
        f32x4 lo = unpack4(((u64)(uint32_t)v[1] << 32) | (uint32_t)v[0]);
        f32x4 hi = unpack4(((u64)(uint32_t)v[3] << 32) | (uint32_t)v[2]);
        lo = lo * pcs[0] + pcb[0];
        hi = hi * pcs[1] + pcb[1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          lo[e] = lo[e] > 0.f ? lo[e] : palp * lo[e];
          hi[e] = hi[e] > 0.f ? hi[e] : palp * hi[e];
        }
        const uint2 pl = pack4(lo), ph = pack4(hi);
        const i32x4 o = i32x4{(int)pl.x, (int)pl.y, (int)ph.x, (int)ph.y};
        asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(o) : "memory");
      }
    }
  };
  if constexpr (PRE) {
    // step 0's rows: its DMA of every wave landed, transformed before the loop
    wait_vm_barrier_c<(D - 1) * DMAW < 63 ? (D - 1) * DMAW : 63>();
    pre_rows(cp, cslot);
  }
  // Stagger: waves w and w + 4 share a SIMD.  The "late" half runs the
  // epilogue of step v - 1 right after the barrier of step v and then the
  // MFMAs of step v, while the early half runs MFMAs then epilogue of step v:
  // on every SIMD one wave's epilogue / DMA issue / loop control overlaps
  // the other's MFMAs, with one barrier per step and no extra registers
  // (acc of v - 1 is consumed before the MFMAs of v overwrite it).
  const bool late = STAG && wv >= 4;
  // vmcnt accounting, ops younger than DMA(v) (issued in iteration v - D):
  //   early, iteration u: E(u) DMA(u+D) S(u)
  //     -> (D-1) M + S c(v-D) + (E+S) sum_{v-D<u<v} c(u)
  //   late, iteration u: S(u-1) E(u) DMA(u+D)
  //     -> (D-1) M + S sum_{v-D<=u<=v-2} c(u) + E sum_{v-D<u<v} c(u)
  unsigned hist = 0;                            // bit j: iteration v-1-j computed
  constexpr unsigned FULL = (1u << D) - 1;
  constexpr int YE = (D - 1) * DMAW + S + (E + S) * (D - 1);      // steady state, early
  constexpr int YL = (D - 1) * DMAW + S * (D - 1) + E * (D - 1);  // steady state, late
  // F_PRE waits for DMA(v + 1): (D-2) M + S c(v+1-D) + (E+S) sum_{v+1-D<u<v} c(u)
  constexpr unsigned FULLP = (1u << (D - 1)) - 1;
  constexpr int YP = (D - 2) * DMAW + S + (E + S) * (D - 2);
  long long ppix = 0;                           // late half: the step whose epilogue is pending
  int prowg = 0, pxs = 0;
  bool pcomp = false;
  [[maybe_unused]] unsigned long long st_a = 0, st_b = 0, st_wait = 0, st_issue = 0, st_mfma = 0, st_epi = 0,
                                      st_steps = 0, st_t0 = 0, st_t1 = 0;
  S3_STAMP(st_t0);
#pragma unroll 1
  while (cp.c < cend) {
    S3_STAMP(st_a);
    if constexpr (PRE) {
      static_assert(D >= 2 && !STAG, "one step ahead");
      if ((hist & FULLP) == FULLP) {
        wait_vm_barrier_c<YP < 63 ? YP : 63>();
      } else {
        const int y = (D - 2) * DMAW + (((hist >> (D - 2)) & 1) ? S : 0) +
                      (E + S) * __builtin_popcount(hist & ((1u << (D - 2)) - 1));
        wait_vm_barrier(y);
      }
    } else if ((hist & FULL) == FULL) {
      if (late) wait_vm_barrier_c<YL < 63 ? YL : 63>();
      else wait_vm_barrier_c<YE < 63 ? YE : 63>();
    } else {
      const unsigned inner = hist & ((1u << (D - 1)) - 1);          // c(v-1) .. c(v-D+1)
      const int y = late ? (D - 1) * DMAW + S * __builtin_popcount((hist >> 1) & ((1u << (D - 1)) - 1)) +
                               E * __builtin_popcount(inner)
                         : (D - 1) * DMAW + (((hist >> (D - 1)) & 1) ? S : 0) +
                               (E + S) * __builtin_popcount(inner);
      wait_vm_barrier(y);
    }
    S3_STAMP(st_b);
    st_wait += st_b - st_a;
    st_a = st_b;
    const bool comp = cp.kind == S3_COMP;
    const int rowg = cp.img * H + cp.y0;
    const long long pix0 = (long long)rowg * IW + cp.xs;
    if (late && pcomp) epilogue(ppix, prowg, pxs);   // its loads were waited for last iteration
    // epilogue loads BEFORE this iteration's DMA (see the vmcnt accounting)
    if constexpr (E > 0) {
      if (comp) load_e(pix0);
    }
    __builtin_amdgcn_sched_barrier(0);
    issue(lslot, ld, ld.c < cend);
    advance(ld);
    lslot += RPS;
    lslot = lslot >= RING ? lslot - RING : lslot;
    __builtin_amdgcn_sched_barrier(0);
    S3_STAMP(st_b);
    st_issue += st_b - st_a;
    st_a = st_b;
    if (comp) {
      mfma_step(cslot);
      S3_STAMP(st_b);
      st_mfma += st_b - st_a;
      st_a = st_b;
      ++st_steps;
      // wait for the epilogue loads in the iteration that issued them: the
      // compiler does not know the asm loads are asynchronous, so their
      // registers must not be live across the loop back-edge (it may copy
      // them there before the data has landed)
      wait_e();
      if constexpr (SC) {
        // + the 1x1 dgrad of the second gradient (after the 9 taps: the
        // fp32 sum in one order, bitwise-reproducible)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int mi = 0; mi < MC; ++mi)
#pragma unroll
            for (int ni = 0; ni < MP; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  wsr[mi][kb], __builtin_bit_cast(bf16x8, esc[ni][kb]), acc[mi][ni], 0, 0, 0);
      }
      if (!late) epilogue(pix0, rowg, cp.xs);
      S3_STAMP(st_b);
      st_epi += st_b - st_a;
    }
    if constexpr (PRE) {
      Cur nx = cp;
      advance(nx);
      int ncs = cslot + RPS;
      ncs = ncs >= RING ? ncs - RING : ncs;
      if (nx.c < cend) pre_rows(nx, ncs);
    }
    ppix = pix0;
    prowg = rowg;
    pxs = cp.xs;
    pcomp = comp;
    cslot += RPS;
    cslot = cslot >= RING ? cslot - RING : cslot;
    hist = (hist << 1) | (comp ? 1u : 0u);
    advance(cp);
  }
  if (late && pcomp) epilogue(ppix, prowg, pxs);   // the late half's last epilogue
#ifdef RR_S3_STAMPS
  S3_STAMP(st_t1);
  if (lane == 0) {
    unsigned long long *o = rr_s3_stamps + ((long long)blockIdx.x * 8 + wv) * 8;
    o[0] = st_t1 - st_t0; o[1] = st_wait; o[2] = st_issue; o[3] = st_mfma; o[4] = st_epi; o[5] = st_steps;
    o[6] = 1;
  }
#endif
  // drain the ring's trailing (dummy) DMA before the LDS is reused / released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- per-workgroup partials: lanes of one channel (frow) -> waves (wp) ----
  if constexpr (STATS || BNBWD) {
#pragma unroll
    for (int mi = 0; mi < MC; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        {
          r0[mi][j] = row16_sum(r0[mi][j]);
          r1[mi][j] = row16_sum(r1[mi][j]);
        }
    float *red = reinterpret_cast<float *>(smem);   // [4 wp][64][2] + [8 waves]
    if (frow == 0) {
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = wc * 32 + mi * 16 + fq * 4 + j;
          red[(wp * 64 + c) * 2 + 0] = r0[mi][j];
          red[(wp * 64 + c) * 2 + 1] = r1[mi][j];
        }
    }
    if constexpr (BNBWD) {
      ra = wave_sum(ra);
      if (lane == 0) red[4 * 64 * 2 + wv] = ra;
    }
    __syncthreads();
    if (tid < 64) {
      float x = 0.f, y = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        x += red[(q * 64 + tid) * 2 + 0];
        y += red[(q * 64 + tid) * 2 + 1];
      }
      if constexpr (BNBWD) {
        float *pp = a.bpart + ((long long)blockIdx.x * 64 + tid) * 3;
        pp[0] = x;
        pp[1] = a.binv[tid] * (y - a.bmean[tid] * x);
        pp[2] = 0.f;
      } else {
        a.stats[((long long)blockIdx.x * 64 + tid) * 2 + 0] = x;
        a.stats[((long long)blockIdx.x * 64 + tid) * 2 + 1] = y;
      }
    }
    if constexpr (BNBWD) {
      if (tid == 0) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) s += red[4 * 64 * 2 + q];
        a.bapart[blockIdx.x] = s;
      }
    }
  }
}

// epilogue flag set of a call, or -1 when the streaming kernel has no
// instance for it (the tiled kernel takes the call)
int s3_flags(const rr_igemm_desc *d, bool bnbwd) {
  if (bnbwd) return F_BNBWD;
  const int f = (d->has_bias ? F_BIAS : 0) | (d->want_stats ? F_STATS : 0) |
                (d->act == RR_ACT_RELU ? F_RELU : 0) | (d->accumulate ? F_ACC : 0) |
                (d->has_mask ? F_MASK : 0);
  switch (f) {
    case 0: case F_BIAS: case F_STATS: case F_BIAS | F_STATS: case F_RELU: case F_BIAS | F_RELU:
    case F_ACC: case F_MASK: case F_ACC | F_MASK:
      return f;
    default:
      return -1;
  }
}

template <int W, int MP, int F, int STG = -1, bool SM = false>
void launch1(const S3Args &a, int P, hipStream_t st) {
  // the late-epilogue stagger measured faster only for 256-pixel steps
  // without the BN-statistics registers (it keeps acc live across the loop
  // back-edge: the stats variants spill with it)
  constexpr int STAG = STG >= 0 ? STG : ((MP == 4 && !(F & F_STATS)) ? 1 : 0);
  hipLaunchKernelGGL((stream3_kernel<W, MP, F, STAG, SM>), dim3(S3_WG), dim3(512), 0, st, a, P / (64 * MP));
}

template <int W>
int launch_w(const S3Args &a, int f, int P, hipStream_t st) {
  // the dgrad (no epilogue) and the bias + ReLU forward in 128-pixel steps
  // too: in the graph-captured step they beat the staggered 256-pixel form
  // by 0.8 % (profiles/r3an_ab_s3_mp4.txt; the stagger had been measured
  // faster on eager launches)
  switch (f) {
    case 0: launch1<W, 2, 0, 0>(a, P, st); break;
    case F_BIAS | F_RELU: launch1<W, 2, F_BIAS | F_RELU, 0>(a, P, st); break;
    case F_BIAS: launch1<W, 4, F_BIAS>(a, P, st); break;
    // the BN-statistics forward in 128-pixel steps: with 256-pixel steps the
    // statistics registers pushed the kernel past 256 VGPRs (10 spilled at
    // W = 64, 26 at W = 32: scratch traffic in the step loop, 224 us vs 139
    // us for the non-statistics 64x64 forward); 128-pixel steps fit in 220
    // (graph step +1.3 %, profiles/r3am_ab_s3_stats.txt)
    case F_STATS: launch1<W, 2, F_STATS, 0>(a, P, st); break;
    case F_BIAS | F_STATS: launch1<W, 2, F_BIAS | F_STATS, 0>(a, P, st); break;
    case F_RELU: launch1<W, 4, F_RELU>(a, P, st); break;
    case F_ACC: launch1<W, 2, F_ACC>(a, P, st); break;
    case F_MASK: launch1<W, 2, F_MASK>(a, P, st); break;
    case F_ACC | F_MASK: launch1<W, 2, F_ACC | F_MASK>(a, P, st); break;
    case F_BNBWD: launch1<W, 2, F_BNBWD>(a, P, st); break;
    case F_BIAS | F_STATS | F_PRE: launch1<W, 2, F_BIAS | F_STATS | F_PRE, 0>(a, P, st); break;
    // the eval epilogues (stream3_launch_ex), 128-pixel steps
    case F_BIAS | F_PRELU: launch1<W, 2, F_BIAS | F_PRELU, 0>(a, P, st); break;
    case F_BIAS | F_RES | F_RELU: launch1<W, 2, F_BIAS | F_RES | F_RELU, 0>(a, P, st); break;
    case F_BIAS | F_RES | F_RELU | F_POOL | F_PFULL | F_PNOIDX:
      launch1<W, 2, F_BIAS | F_RES | F_RELU | F_POOL | F_PFULL | F_PNOIDX, 0>(a, P, st); break;
    case F_BIAS | F_RELU | F_POOL | F_PFULL | F_PNOIDX:
      launch1<W, 2, F_BIAS | F_RELU | F_POOL | F_PFULL | F_PNOIDX, 0>(a, P, st); break;
    case F_BIAS | F_RELU | F_POOL | F_PNOIDX: launch1<W, 2, F_BIAS | F_RELU | F_POOL | F_PNOIDX, 0>(a, P, st); break;
    default: return RR_EUNSUPPORTED;
  }
  RR_CHECK_LAUNCH();
  return RR_OK;
}

// column-strip mode: the flag sets it has instances for -- the plain conv /
// dgrad, bias (+ ReLU), and the BN-folded eval epilogues of the reference's
// 224 pipeline (17:84-86, 18:46-47); the training epilogues (statistics,
// operands, BN backward, the window index) stay on the tap-reuse conv there
bool s3_strip_flags(int f) {
  switch (f) {
    case 0: case F_BIAS: case F_BIAS | F_RELU: case F_BIAS | F_PRELU: case F_BIAS | F_RES | F_RELU:
    case F_BIAS | F_RES | F_RELU | F_POOL | F_PFULL | F_PNOIDX:
    case F_BIAS | F_RELU | F_POOL | F_PFULL | F_PNOIDX:
    case F_BIAS | F_RELU | F_POOL | F_PNOIDX:
      return true;
    default:
      return false;
  }
}

int launch_strips(const S3Args &a, int f, int P, hipStream_t st) {
  // 32-wide strips, 128-pixel steps (4 rows), no stagger
  switch (f) {
    case 0: launch1<32, 2, 0, 0, true>(a, P, st); break;
    case F_BIAS: launch1<32, 2, F_BIAS, 0, true>(a, P, st); break;
    case F_BIAS | F_RELU: launch1<32, 2, F_BIAS | F_RELU, 0, true>(a, P, st); break;
    case F_BIAS | F_PRELU: launch1<32, 2, F_BIAS | F_PRELU, 0, true>(a, P, st); break;
    case F_BIAS | F_RES | F_RELU: launch1<32, 2, F_BIAS | F_RES | F_RELU, 0, true>(a, P, st); break;
    case F_BIAS | F_RES | F_RELU | F_POOL | F_PFULL | F_PNOIDX:
      launch1<32, 2, F_BIAS | F_RES | F_RELU | F_POOL | F_PFULL | F_PNOIDX, 0, true>(a, P, st); break;
    case F_BIAS | F_RELU | F_POOL | F_PFULL | F_PNOIDX:
      launch1<32, 2, F_BIAS | F_RELU | F_POOL | F_PFULL | F_PNOIDX, 0, true>(a, P, st); break;
    case F_BIAS | F_RELU | F_POOL | F_PNOIDX:
      launch1<32, 2, F_BIAS | F_RELU | F_POOL | F_PNOIDX, 0, true>(a, P, st); break;
    default: return RR_EUNSUPPORTED;
  }
  RR_CHECK_LAUNCH();
  return RR_OK;
}

// column width of the streaming kernel on a w-wide map: the whole row at w =
// 32 / 64, else 32-pixel column strips (the reference's 224 maps: 7 strips;
// a strip's neighbour columns are its halo, read again by the next strip --
// 34 / 32 of the input), 0: not taken
int s3_col(int w) {
  if (w == 32 || w == 64) return w;
  if (w > 64 && w % 32 == 0) return 32;
  return 0;
}

bool s3_is_strip(const rr_igemm_desc *d) { return s3_col(d->w) != d->w; }

// launch flag set f of *d: whole rows or strips
int s3_go(const rr_igemm_desc *d, const S3Args &a, int f, int P, hipStream_t st) {
  if (s3_is_strip(d)) return launch_strips(a, f, P, st);
  if (d->w == 64) return launch_w<64>(a, f, P, st);
  return launch_w<32>(a, f, P, st);
}

}  // namespace

int stream3_geom_ok(const rr_igemm_desc *d) {
  // RR_PATH stream3=0: the tap-reuse / halo kernels instead (tests)
  if (!rr_path("stream3", 1)) return 0;
  if (d->dtype != RR_BF16 || d->mode != RR_CONV3X3) return 0;
  if (d->c_in1 != 64 || d->c_out != 64 || d->out_split || d->out_nchw) return 0;
  const int cw = s3_col(d->w);
  // column strips: RR_PATH stream3_strips=0 leaves the wide maps to the
  // tap-reuse conv's row-segment tiles
  if (!cw || (cw != d->w && !rr_path("stream3_strips", 1))) return 0;
  // eligibility independent of the step size: whole 256-pixel steps (the
  // larger one) and at least one per workgroup
  if (d->h % (256 / cw)) return 0;
  const long long P = (long long)d->n * d->h * d->w;
  // (every element offset is 64-bit: the cfg5 chunks of 1024 224x224 images
  // are 6.6 GB per tensor)
  if (P < 256LL * S3_WG || P > INT_MAX / 2) return 0;
  return S3_WG;
}

int stream3_blocks(const rr_igemm_desc *d, int bnbwd) {
  if (!stream3_geom_ok(d)) return 0;
  // (a concat input, dec1's 64 + 64 -> 64, goes to the tap-reuse conv in
  // one pass with the whole K = 1152 sum in fp32: the same graph-step time
  // as two streaming passes, profiles/r4j_abstep_concat_splitdgrad.txt,
  // without a bf16 rounding of the half sum)
  const int f = s3_flags(d, bnbwd != 0);
  if (d->c_in2 != 0 || f < 0 || (s3_is_strip(d) && !s3_strip_flags(f))) return 0;
  return S3_WG;
}

int stream3_strips(const rr_igemm_desc *d) { return stream3_geom_ok(d) && s3_is_strip(d); }

const char *stream3_name(const rr_igemm_desc *d, const char *suffix) {
  static const char *names[4][5] = {
      {"stream3_kernel<64>", "stream3_kernel<64,pool>", "stream3_kernel<64,sc>", "stream3_kernel<64,ex>", "stream3_kernel<64,bnbwd>"},
      {"stream3_kernel<32>", "stream3_kernel<32,pool>", "stream3_kernel<32,sc>", "stream3_kernel<32,ex>", "stream3_kernel<32,bnbwd>"},
      {"stream3_kernel<s64>", "stream3_kernel<s64,pool>", "stream3_kernel<s64,sc>", "stream3_kernel<s64,ex>", "stream3_kernel<s64,bnbwd>"},
      {"stream3_kernel<s32>", "stream3_kernel<s32,pool>", "stream3_kernel<s32,sc>", "stream3_kernel<s32,ex>", "stream3_kernel<s32,bnbwd>"}};
  const int cw = s3_col(d->w);
  const int r = (cw == d->w ? 0 : 2) + (cw == 64 ? 0 : 1);   // (strips: 32 wide)
  int c = 0;
  if (suffix && suffix[0]) {
    switch (suffix[0]) {
      case 'p': c = 1; break;
      case 's': c = 2; break;
      case 'e': c = 3; break;
      default: c = 4; break;
    }
  }
  return names[r][c];
}

// the eval flag set of an rr_igemm_ex call, or -1
static int s3_ex_flags(const rr_igemm_desc *d) {
  if (!d->has_bias || d->want_stats || d->accumulate || d->has_mask) return -1;
  const int act = d->act;
  const bool prelu = (act & 3) == RR_ACT_PRELU, relu = (act & 3) == RR_ACT_RELU;
  const bool res = (act & RR_ACT_RES) != 0, pool = (act & RR_ACT_POOL) != 0, full = !(act & RR_ACT_NOFULL);
  if (prelu) return res || pool ? -1 : F_BIAS | F_PRELU;
  if (!relu) return -1;
  if (res && !pool) return F_BIAS | F_RES | F_RELU;
  if (res && pool && full) return F_BIAS | F_RES | F_RELU | F_POOL | F_PFULL | F_PNOIDX;
  if (!res && pool) return F_BIAS | F_RELU | F_POOL | F_PNOIDX | (full ? F_PFULL : 0);
  return -1;
}

int stream3_ex_ok(const rr_igemm_desc *d) {
  if (!stream3_geom_ok(d) || d->c_in2 != 0) return 0;
  if ((d->act & RR_ACT_POOL) && (d->h % 2 || d->w % 2)) return 0;
  return s3_ex_flags(d) >= 0 ? S3_WG : 0;
}

int stream3_launch_ex(const rr_igemm_desc *d, const S3Args &a0, hipStream_t st) {
  const int f = s3_ex_flags(d);
  if (!stream3_ex_ok(d) || f < 0 || !a0.x || !a0.wt || !a0.bias || ((f & F_PRELU) && !a0.alpha) ||
      ((f & F_RES) && !a0.res) || ((f & F_POOL) && !a0.ypool) || (((f & F_PFULL) || !(f & F_POOL)) && !a0.y))
    return RR_EUNSUPPORTED;
  S3Args a = a0;
  a.wld = 64; a.woff = 0; a.w = d->w;
  const int P = d->n * d->h * d->w;
  return s3_go(d, a, f, P, st);
}

#ifdef RR_S3_STAMPS
extern "C" int rr_s3_stamps_read(unsigned long long *host, int n, int clear) {
  if (n > 256 * 8 * 8) n = 256 * 8 * 8;
  if (host && hipMemcpyFromSymbol(host, HIP_SYMBOL(rr_s3_stamps), (size_t)n * 8) != hipSuccess) return -3;
  if (clear) {
    static unsigned long long z[256 * 8 * 8];
    if (hipMemcpyToSymbol(HIP_SYMBOL(rr_s3_stamps), z, sizeof(z)) != hipSuccess) return -3;
  }
  return 0;
}
#endif

int stream3_launch_sc(const rr_igemm_desc *d, const S3Args &a0, hipStream_t st) {
  if (!stream3_blocks(d, 0) || d->c_in2 || s3_flags(d, false) != 0 || !a0.xsc || !a0.wsc || s3_is_strip(d))
    return RR_EUNSUPPORTED;
  S3Args a = a0;
  a.wld = 64; a.woff = 0; a.w = d->w;
  const int P = d->n * d->h * d->w;
  // 128-pixel steps, no stagger (the plain dgrad's form, launch_w)
  if (d->w == 64) launch1<64, 2, F_SC, 0>(a, P, st);
  else launch1<32, 2, F_SC, 0>(a, P, st);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

int stream3_launch_pool(const rr_igemm_desc *d, const S3Args &a0, hipStream_t st) {
  if (!stream3_blocks(d, 0) || d->c_in2 || d->act != RR_ACT_RELU || d->accumulate || d->has_mask ||
      d->want_stats || !a0.ypool || (!a0.pidx && !d->has_bias) || (a0.pidx && s3_is_strip(d)))
    return RR_EUNSUPPORTED;
  S3Args a = a0;
  a.wld = 64; a.woff = 0; a.w = d->w;
  const int P = d->n * d->h * d->w;
  if (!a0.pidx)   // (the eval judge: no window index)
    return s3_go(d, a, F_BIAS | F_RELU | F_POOL | F_PNOIDX, P, st);
  // 128-pixel steps, no stagger: the bias + ReLU forward's form (launch_w;
  // 256-pixel steps at W = 64 were bitwise equal and within the run order's
  // noise, profiles/r5zi_pool_bench.jsonl, r5zj_pool_bench.jsonl)
  if (d->w == 64) {
    if (d->has_bias) launch1<64, 2, F_BIAS | F_RELU | F_POOL, 0>(a, P, st);
    else launch1<64, 2, F_RELU | F_POOL, 0>(a, P, st);
  } else {
    if (d->has_bias) launch1<32, 2, F_BIAS | F_RELU | F_POOL, 0>(a, P, st);
    else launch1<32, 2, F_RELU | F_POOL, 0>(a, P, st);
  }
  RR_CHECK_LAUNCH();
  return RR_OK;
}

int stream3_launch_pre(const rr_igemm_desc *d, const S3Args &a0, hipStream_t st) {
  if (!stream3_blocks(d, 0) || s3_is_strip(d) || s3_flags(d, false) != (F_BIAS | F_STATS) || !a0.pre_s ||
      !a0.pre_b || !a0.pre_alpha)
    return RR_EUNSUPPORTED;
  S3Args a = a0;
  a.wld = 64; a.woff = 0; a.w = d->w;
  const int P = d->n * d->h * d->w;
  if (d->w == 64) return launch_w<64>(a, F_BIAS | F_STATS | F_PRE, P, st);
  return launch_w<32>(a, F_BIAS | F_STATS | F_PRE, P, st);
}

int stream3_launch(const rr_igemm_desc *d, const S3Args &a0, int bnbwd, hipStream_t st) {
  if (!stream3_blocks(d, bnbwd)) return RR_EUNSUPPORTED;
  S3Args a = a0;
  const int P = d->n * d->h * d->w;
  a.wld = 64; a.woff = 0; a.w = d->w;
  const int f = s3_flags(d, bnbwd != 0);
  return s3_go(d, a, f, P, st);
}
