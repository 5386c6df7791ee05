// conv3r.hip -- tap-reuse 3x3 bf16 convolution: forward, dgrad and the
// fused BN/PReLU-backward dgrad of the 64-512-channel layers on 8x8, 16x16
// and 32x32 maps (ResUNet res2 / res3 / dec2 / dec3 / bottleneck,
// 14_train_unified_advanced.py:96-186; VGG16 conv2_x / conv3_x of the
// perceptual loss, 14:189-196; SimpleUNet enc2 / bottleneck / dec2,
// 07:75-120).
//
// What bounds the LDS-halo igemm (igemm.hip) on these layers is the LDS
// port: its 8 waves own 64 x 32 output tiles and re-read a 64 x 64 weight
// stage and a 32-pixel activation stage from LDS for every 16 MFMAs, ~768 B
// of fragment reads per MFMA against the ~1 KB the port supplies per MFMA
// slot, and every (K chunk, tap) stage ends in a barrier.  Here a wave owns
// 128 output pixels = R whole output rows (W = 16, 32) or the same 8 rows of
// two images (W = 8), times 64 output channels, and walks the K loop in
// stages of (32 input channels, tap column dx):
//
//   * the halo of the tile (its rows + 1 above / below, zero at the image
//     edges) for 32 input channels sits in LDS as 1-KB blocks of 16 pixels x
//     4 channel planes of 8 (block byte = plane * 256 + pixel * 16), so a
//     B-fragment read (ds_read_b128: lane = pixel l & 15, plane l >> 4) of
//     16 consecutive pixels at ANY shift hits 16 distinct bank slots;
//   * per stage the wave loads the A fragments (weights) of the three taps
//     (dy, dx), dy = 0..2, once (12 reads), then streams its R + 2 halo rows:
//     halo row ri is read ONCE and feeds output rows ri, ri - 1, ri - 2 (taps
//     dy = 0, 1, 2) -- 3 x NM MFMAs per fragment read instead of NM;
//   * the left / right zero padding is not stored: the shifted read of the
//     edge column is zeroed in registers (one v_cndmask per dword);
//   * 96 MFMAs per wave per stage (R x NS x NM x 3), one barrier per stage;
//     LDS fragment traffic ~240 B per MFMA;
//   * operands arrive by LDS-DMA (global_load_lds_dwordx4) one stage ahead
//     into double buffers: the next stage's weights (the 1-KB tiles the pack
//     writes behind the [c_out][9][c_in] rows, rr_pack_conv: a stage is 3
//     contiguous runs of whole lines -- gathered from the row layout as
//     64-B pieces it cost ~14% of the kernel) and, at the first stage of a chunk, the next
//     chunk's halo (from the NHWC activations; out-of-image rows from the
//     zero page).  hipcc would drain the DMA (vmcnt(0)) before any ds_read
//     it cannot separate from a DMA destination, so the fragment reads are
//     inline asm with counted lgkmcnt waits, and the stage boundary is a
//     counted vmcnt + raw s_barrier;
//   * the epilogue stages one 128-pixel group at a time as fp32 [128][BC]
//     in LDS and reuses the tiled kernels' staged store (igemm_epi.h): BN
//     statistics (one partial row per 128 pixels), bias, ReLU, accumulate,
//     ReLU-backward mask, concat split, or the fused BN/PReLU backward.
//
// Workgroup: 8 waves = WC channel groups x WP pixel groups; BC = 64 NW
// channels per wave group.  Geometry per (W, BC) in R3 below.
#include "common.h"
#include "conv3r.h"

#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace {

template <int W, int BC, int NW, int NWV, int HB, int SG> struct R3 {
  // SG > 0: row-segment tiles of any H x W (W ignored): TR rows x 16 SG
  // columns of one image; out-of-image rows / columns are zero in the halo
  // and masked in the epilogue
  static constexpr bool SEGM = SG > 0;
  static constexpr bool PAIR = !SEGM && W == 8;     // a row unit = the same row of 2 images
  static constexpr int NS = SEGM ? SG : (PAIR ? 1 : W / 16);   // 16-pixel column blocks per row unit
  static constexpr int R = SEGM ? 8 / SG : (PAIR ? 8 : 128 / W);  // output rows per wave
  static constexpr int NM = NW / 16;                // 16-channel MFMA rows per wave
  static constexpr int NT = 64 * NWV;               // threads per workgroup
  static constexpr int WC = BC / NW, WP = NWV / WC; // wave grid
  static constexpr int TPX = WP * 128;              // pixels per tile
  static constexpr int TR = PAIR ? 8 : WP * R;      // tile rows (W >= 16)
  static constexpr int HS = PAIR ? 8 : (SEGM || TR < W ? TR : W);        // output rows per halo segment
  static constexpr int SEG = PAIR ? WP : (SEGM || TR < W ? 1 : TR / W);  // segments (images / pairs)
  static constexpr int HROWS = SEG * (HS + 2);
  // blocks per halo row: a row-segment tile keeps a side block in front of
  // each row -- slot 15 = the pixel left of the segment, slot 0 = the pixel
  // right of the previous row's segment -- so the shifted edge reads land on
  // real neighbours (or zeros) with no register fix-up; one trailing side
  // block serves the last row
  static constexpr int RS = SEGM ? NS + 1 : NS;
  static constexpr int HBLK = SEGM ? HROWS * RS + 1 : HROWS * NS;  // 1-KB halo blocks per chunk
  static constexpr int HBYTES = HBLK * 1024;
  static constexpr int WBLK = 3 * (BC / 16);        // weight blocks per stage (3 taps)
  static constexpr int WBYTES = WBLK * 1024;
  static constexpr int NHG = (HBLK + NWV - 1) / NWV;   // halo DMA pieces per wave per chunk
  static constexpr int NWG = (WBLK + NWV - 1) / NWV;   // weight DMA pieces per wave per stage
  static constexpr int SROW = BC + 4;
  static constexpr int STG = 128 * SROW * 4 + (NWV * BC * 2 + NWV) * 4 + 256;
  // [weights x2][halo x HB][guard block]: the shifted edge reads stay inside
  // (row-segment tiles read inside their side blocks: no guard)
  static constexpr int HOFF = 2 * WBYTES;                        // halo base
  static constexpr int KBYTES = 2 * WBYTES + HB * HBYTES + (SEGM ? 0 : 1024);
  static constexpr int BIAS = KBYTES;               // [BC] fp32 bias for the register epilogue
  static constexpr int LDS = KBYTES + BC * 4 > STG || SEGM ? KBYTES + BC * 4 : STG;
  static_assert(LDS <= 160 * 1024 && (NWV != 4 || 2 * LDS <= 160 * 1024), "LDS");
  static_assert(WC * WP == NWV && NM * 16 == NW, "wave grid");
  static_assert(HB == 1 || HB == 2, "halo buffers");
  static_assert(!SEGM || (SG == 1 || SG == 2), "segment width");
  static_assert(SEGM || PAIR || TR % W == 0 || W % TR == 0, "tile rows");
  static_assert(2 * WBYTES >= 1024, "the edge read of the first halo block stays in LDS");
  static_assert(2 * NM + NS <= 15, "lgkmcnt of the row-0 wait");
};

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int N> __device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

#ifdef RR_CONV3R_STAMPS
// diagnostic build only (make stamps; tools/conv3r_stamps.py): per-wave sums
// of the K loop's segments, read with rr_conv3r_stamps; never shipped
__device__ unsigned long long rr_c3_stamps[1 << 18];
#define C3_STAMP(t)                                                              \
  do {                                                                          \
    __builtin_amdgcn_sched_barrier(0);                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");   \
    __builtin_amdgcn_sched_barrier(0);                                          \
  } while (0)
template <int N> __device__ __forceinline__ void vm_barrier_st(unsigned long long &tw, unsigned long long &tb) {
  unsigned long long t0, t1, t2;
  C3_STAMP(t0);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  C3_STAMP(t1);
  asm volatile("s_barrier" ::: "memory");
  C3_STAMP(t2);
  tw += t1 - t0;
  tb += t2 - t1;
}
#define VM_BARRIER(N) vm_barrier_st<N>(st_vm, st_bar)
// the wave's epilogue time (K loop end -> any return), written at scope exit
struct C3EpiStamp {
  unsigned long long *o = nullptr;
  unsigned long long t1 = 0;
  __device__ ~C3EpiStamp() {
    if (o) {
      unsigned long long t;
      C3_STAMP(t);
      o[7] = t - t1;
    }
  }
};
#else
#define C3_STAMP(t) do {} while (0)
#define VM_BARRIER(N) vm_barrier<N>()
#endif

template <int N> using ic = std::integral_constant<int, N>;

// EPI: 0 = every epilogue (operand loads: accumulate / residual / ReLU mask,
// PReLU, pool, the fused BN backward), 1 = bias, statistics, ReLU and the
// concat split only -- the forward and plain dgrad of the training step,
// 2 = 1 + the accumulate / ReLU-mask operands (the identity-shortcut and VGG
// dgrads), 3 = the fused BN -> PReLU backward only, 4 = 1 + the 2x2 max-pool
// (the perceptual VGG's conv + ReLU + MaxPool2d, rr_igemm_pool), 5 = 4 + the
// residual and PReLU (the BN-folded eval forward of the restore path,
// rr_igemm_ex: the general instance sat at 256 VGPRs with scratch spills on
// the row-segment tiles of the cfg5 geometry).  A specialised instance
// holds no registers for the epilogues it cannot run (no spills) and carries
// none of their branches: the plain epilogue's instruction stream is a third
// of the general one's (989 vs the general path's share of 11.7 k).
template <int W, int BC, int NW, int NWV, int HB, int SG, int EPI = 0>
__global__ __launch_bounds__(64 * NWV, 8 / NWV) void conv3r_kernel(IgemmArgs a) {
  using G = R3<W, BC, NW, NWV, HB, SG>;
  // the fused BN/PReLU-backward dgrad epilogue runs in registers on the
  // row-segment tiles and the 8-wave whole-row tiles (16x16 / 8x8: 1-4 %
  // faster than staging it through the LDS one 128-pixel group at a time,
  // profiles/r5d_ablayers_bnbwd.txt) and in the bnbwd-only instance (EPI 3,
  // spill-free); the general instance stages it on the 4-wave whole-row tiles
  // (32x32: its register form was 12 % slower there)
  constexpr bool BNREG = G::SEGM || NWV == 8 || EPI == 3;
  constexpr bool ALLOW_BN = EPI == 0 || EPI == 3;     // the fused BN backward (a.bpart)
  constexpr bool ALLOW_OPS = EPI == 0 || EPI == 2;    // accumulate / ReLU-mask operands
  constexpr bool ALLOW_EX = EPI == 0 || EPI == 5;     // residual, PReLU
  constexpr bool ALLOW_POOL = EPI == 0 || EPI == 4 || EPI == 5;   // the 2x2 max-pool epilogue
  constexpr int NS = G::NS, R = G::R, NM = G::NM, WC = G::WC, RS = G::RS;
  constexpr int HW = W * W;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  [[maybe_unused]] unsigned long long st_k0 = 0;
  C3_STAMP(st_k0);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wv % WC, wp = wv / WC;
  const int frow = lane & 15, fq = lane >> 4;

  // XCD-aware tile order (as igemm3_halo_kernel): XCD b % 8 walks a
  // contiguous tile range, so column blocks of a pixel tile share its L2
  int tile = blockIdx.x;
  if (a.xcd) {
    const int per = (int)gridDim.x / 8;
    if ((int)blockIdx.x < per * 8) tile = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
  }
  const int cblk = tile % a.ncblk, pblk = tile / a.ncblk;
  const int c0 = cblk * BC;
  const int p0 = pblk * G::TPX;
  int n0, ys, xs = 0;                                // image, first tile row / column
  if constexpr (G::SEGM) {
    // pixel tile = (image, row band, column segment), segments fastest
    const int nseg = (a.w + 16 * NS - 1) / (16 * NS), nband = (a.h + G::TR - 1) / G::TR;
    const int seg = pblk % nseg, t2 = pblk / nseg;
    const int band = t2 % nband;
    n0 = t2 / nband;
    ys = band * G::TR;
    xs = seg * 16 * NS;
  } else {
    n0 = p0 / HW;
    ys = G::PAIR || G::TR >= W ? 0 : (p0 - n0 * HW) / W;   // (one segment)
  }

  const uint32_t sbase = (uint32_t)(uintptr_t)smem;
  const uint32_t wbase = sbase, hbase = sbase + G::HOFF;

  // ---- per-lane DMA sources ----
  // halo block b = (segment k, halo row hr, column block s): pixel index of
  // this lane's 16 B (-1: zero padding row)
  int hpix[G::NHG], hdst[G::NHG];
#pragma unroll
  for (int i = 0; i < G::NHG; ++i) {
    int b = wv + NWV * i;
    if (b >= G::HBLK) b -= NWV;                     // a duplicate of this wave's previous block
    const int k = b / ((G::HS + 2) * RS);
    const int rem = b - k * ((G::HS + 2) * RS);
    const int hr = rem / RS, s = rem - (rem / RS) * RS;
    int pix = -1;
    if constexpr (G::SEGM) {
      // s = 0: side block (slot 15: left of row hr; slot 0: right of row
      // hr - 1); s >= 1: columns 16 (s - 1) .. of row hr (one segment: the
      // trailing side block is row HS + 2)
      const int hr_ = b / RS, s_ = b - hr_ * RS;
      int y = ys + hr_ - 1, x = -1;
      if (s_ > 0) x = xs + 16 * (s_ - 1) + frow;
      else if (frow == 15) x = xs - 1;
      else if (frow == 0) { x = xs + 16 * NS; --y; }
      if (x >= 0 && x < a.w && y >= 0 && y < a.h) pix = (n0 * a.h + y) * a.w + x;
    } else if constexpr (G::PAIR) {
      const int y = hr - 1;
      if (y >= 0 && y < W) pix = ((n0 + 2 * k + (frow >> 3)) * W + y) * W + (frow & 7);
    } else {
      const int y = ys + hr - 1;
      if (y >= 0 && y < W) pix = ((n0 + k) * W + y) * W + 16 * s + frow;
    }
    hpix[i] = pix;
    hdst[i] = b * 1024;
  }
  // weight block wb = (tap row dy, 16-channel block m): this lane's row
  int wrow[G::NWG], wdst[G::NWG];
#pragma unroll
  for (int i = 0; i < G::NWG; ++i) {
    int b = wv + NWV * i;
    if (b >= G::WBLK) b -= NWV;
    const int dy = b / (BC / 16), m = b - dy * (BC / 16);
    // (row dy of the stage's 3 runs, block mb of the tiles, this lane's 16 B)
    wrow[i] = (dy * (a.cout / 16) + c0 / 16 + m) * 1024 + lane * 16;
    wdst[i] = b * 1024;
  }
  // the weight tiles follow the [c_out][9][c_in] pack (rr_pack_conv)
  const char *wtile = a.wt + (long long)a.cout * a.K * 2;
  auto issue_w = [&](int st) __attribute__((always_inline)) {
    const int ch = st / 3, dx = st - ch * 3;
    char *dst = smem + (st & 1) * G::WBYTES;
    // tiles (chunk ch, column dx, row dy, block mb): 3 contiguous runs per stage
    const char *wst = wtile + (long long)((ch * 3 + dx) * 3) * (a.cout / 16) * 1024;
#pragma unroll
    for (int i = 0; i < G::NWG; ++i)
      __builtin_amdgcn_global_load_lds((const void *)(wst + wrow[i]), LDS_PTR(dst + wdst[i]), 16, 0, 0);
  };
  auto issue_h = [&](int ch) __attribute__((always_inline)) {
    const int ci0 = ch * 32;
    const bool first = ci0 < a.c1;                  // uniform
    const char *base = first ? a.x1 : a.x2;
    const long long cs = first ? a.c1 : a.c2;
    const long long cl = first ? ci0 : ci0 - a.c1;
    const long long zoff = (long long)((uintptr_t)rr_zero_page - (uintptr_t)base) + fq * 16;
    char *dst = smem + G::HOFF + (HB == 2 ? (ch & 1) * G::HBYTES : 0);
#pragma unroll
    for (int i = 0; i < G::NHG; ++i) {
      const long long off = hpix[i] >= 0 ? ((long long)hpix[i] * cs + cl) * 2 + fq * 16 : zoff;
      __builtin_amdgcn_global_load_lds((const void *)(base + off), LDS_PTR(dst + hdst[i]), 16, 0, 0);
    }
  };

  // ---- fragment addressing ----
  // A: weight block (dy, wc * NM + m) of the stage buffer; the lane reads
  // its 16 B at lane * 16 (plane fq, row frow)
  const uint32_t a_lane = wbase + (wc * NM) * 1024 + lane * 16;
  // B: the wave's first halo row (output row 0 minus 1) ...
  int hrow0;
  if constexpr (G::PAIR) {
    hrow0 = wp * (G::HS + 2);
  } else {
    const int r0 = wp * R;                           // first output row of the wave in the tile
    const int k = r0 / G::HS;
    hrow0 = k * (G::HS + 2) + (r0 - k * G::HS);
  }
  // ... and the lane part of a read at tap column dx (pixel frow + dx - 1)
  uint32_t loff[3];
  bool zl[3];                                        // lane reads a padding column at dx
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    if constexpr (G::PAIR) {
      const int x = (frow & 7) + dx - 1;
      const int xc = x < 0 ? 0 : (x > 7 ? 7 : x);
      loff[dx] = fq * 256 + ((frow >> 3) * 8 + xc) * 16;
      zl[dx] = x != xc;
    } else {
      const int x = frow + dx - 1;                  // -1 / 16: the neighbouring block
      loff[dx] = x < 0 ? fq * 256 + 240 - 1024 : (x > 15 ? fq * 256 + 1024 : fq * 256 + x * 16);
      zl[dx] = !G::SEGM && (x < 0 || x > 15);       // (side blocks hold the neighbours)
    }
  }
  const uint32_t b_wave = hbase + (hrow0 * RS + (G::SEGM ? 1 : 0)) * 1024;

  f32x4 acc[R][NS][NM];
#pragma unroll
  for (int o = 0; o < R; ++o)
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int m = 0; m < NM; ++m) acc[o][s][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the bias of the column block for the register epilogue, read before any
  // DMA is in flight (the compiler's wait for a plain load would drain them)
  float *lbias = reinterpret_cast<float *>(smem + G::BIAS);
  if (!a.bpart && tid < BC) lbias[tid] = a.bias ? a.bias[c0 + tid] : 0.f;
  __builtin_amdgcn_s_waitcnt(0x0F70);               // vmcnt(0) (gfx9 encoding)

  const int kc = a.cin / 32, nst = 3 * kc;
  [[maybe_unused]] unsigned long long st_vm = 0, st_bar = 0, st_row0 = 0, st_loop0 = 0, st_loop1 = 0, st_t = 0;
  C3_STAMP(st_loop0);
#ifdef RR_CONV3R_STAMPS
  C3EpiStamp epi_stamp;
#endif
  // prologue: chunk 0's halo, stage 0's weights
  issue_h(0);
  issue_w(0);
  vm_barrier<0>();

  // (no wave priority around the MFMA clusters: +3.3 % when it was added
  // next to the run-time switches, profiles/r3aa_ab*.jsonl; without them it
  // measured -0.6 % at 224 and -0.2 % on the step, r4zd)
  for (int st = 0; st < nst; ++st) {
    const int ch = st / 3, dx = st - ch * 3;       // uniform
    C3_STAMP(st_t);
    // operands of the next stage (weights) and of the next chunk (halo)
    const bool next_h = HB == 2 && dx == 0 && ch + 1 < kc;
    const bool next_w = st + 1 < nst;
    if (HB == 1 && dx == 0 && ch > 0) {
      // one halo buffer: every wave is past the previous chunk's last read
      // (the barrier that ended the last stage); load this chunk's halo
      issue_h(ch);
      VM_BARRIER(0);
    }

    const uint32_t aa = a_lane + (st & 1) * G::WBYTES;
    const uint32_t ba = b_wave + (HB == 2 ? (ch & 1) * G::HBYTES : 0) +
                        (dx == 0 ? loff[0] : (dx == 1 ? loff[1] : loff[2]));
    const bool zlo = dx == 0 && zl[0];               // left padding column (block s = 0)
    const bool zhi = dx == 2 && zl[2];               // right padding column (block NS - 1)
    // fragment reads in the order the rows need them: row 0 uses only the
    // dy = 0 taps, so A(dy 0) and halo row 0 go first and row 0's MFMAs
    // start after NM + NS reads; A(dy 1, 2) and halo row 1 land behind them
    // (waited for at row 1)
    i32x4 af[3][NM];
    i32x4 bf[2][NS];
    auto read_a = [&](int dy) __attribute__((always_inline)) {
#pragma unroll
      for (int m = 0; m < NM; ++m)
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(af[dy][m]) : "v"(aa), "i"((dy * (BC / 16) + m) * 1024));
    };
    read_a(0);
#pragma unroll
    for (int s = 0; s < NS; ++s)
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bf[0][s]) : "v"(ba), "i"(s * 1024));
    read_a(1);
    read_a(2);
#pragma unroll
    for (int ri = 0; ri < R + 2; ++ri) {
      if (ri + 1 < R + 2) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
          asm volatile("ds_read_b128 %0, %1 offset:%2"
                       : "=v"(bf[(ri + 1) & 1][s]) : "v"(ba), "i"(((ri + 1) * RS + s) * 1024));
        if (ri == 0) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(2 * NM + NS) : "memory");
        else asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NS) : "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) asm volatile("" : "+v"(bf[ri & 1][s]));
      if (ri == 0) {
#pragma unroll
        for (int m = 0; m < NM; ++m) asm volatile("" : "+v"(af[0][m]));
#ifdef RR_CONV3R_STAMPS
        unsigned long long t1;
        C3_STAMP(t1);
        st_row0 += t1 - st_t;
#endif
      }
      if (ri == 1) {
#pragma unroll
        for (int dy = 1; dy < 3; ++dy)
#pragma unroll
          for (int m = 0; m < NM; ++m) asm volatile("" : "+v"(af[dy][m]));
      }
      // the padding columns: zero the shifted edge reads
      if constexpr (!G::SEGM) {
        i32x4 &lo = bf[ri & 1][0];
        i32x4 &hi = bf[ri & 1][NS - 1];
        if (G::PAIR) {
          if (zlo || zhi) lo = i32x4{0, 0, 0, 0};
        } else {
          if (zlo) lo = i32x4{0, 0, 0, 0};
          if (zhi) hi = i32x4{0, 0, 0, 0};
        }
      }
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int o = ri - dy;
        if (o < 0 || o >= R) continue;
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int m = 0; m < NM; ++m)
            acc[o][s][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, af[dy][m]), __builtin_bit_cast(bf16x8, bf[ri & 1][s]),
                acc[o][s][m], 0, 0, 0);
      }
      // the DMA for the next stage / chunk goes out behind the first rows'
      // MFMAs (issued right after the barrier, every wave of a SIMD would
      // sit in ~60-cycle issue slots before its first MFMA); the weights
      // first, the halo (waited for one stage later) last
      if (ri == 0 && next_w) issue_w(st + 1);
      if (ri == 1 && next_h) issue_h(ch + 1);
    }
    // the next stage's weights must have landed; a next chunk's halo (issued
    // after them) may stay in flight for one more stage
    if (next_h) VM_BARRIER(G::NHG);
    else VM_BARRIER(0);
  }
#ifdef RR_CONV3R_STAMPS
  C3_STAMP(st_loop1);
  if (lane == 0 && blockIdx.x < (1 << 18) / (8 * NWV)) {
    unsigned long long *o = rr_c3_stamps + ((long long)blockIdx.x * NWV + wv) * 8;
    o[0] = st_loop1 - st_loop0; o[1] = st_row0; o[2] = st_vm; o[3] = st_bar;
    o[4] = (unsigned long long)nst; o[5] = 1;
    o[6] = st_loop0 - st_k0;                        // prologue (kernel entry -> K loop)
    epi_stamp.o = o;
    epi_stamp.t1 = st_loop1;
  }
#endif

  const int cb = wc * NW;                           // the wave's first column in the block
  const int srow = pblk * G::WP + wp;               // the wave's statistics / partial row
  // output pixel of accumulator tile (o, s) for this lane; -1: outside the
  // image (row-segment tiles)
  auto pix_at = [&](int o, int s) __attribute__((always_inline)) -> long long {
    if constexpr (G::SEGM) {
      const int y = ys + wp * R + o, x = xs + 16 * s + frow;
      return y < a.h && x < a.w ? ((long long)n0 * a.h + y) * a.w + x : -1LL;
    } else {
      return (long long)p0 + wp * 128 +
             (G::PAIR ? (frow >> 3) * 64 + o * 8 + (frow & 7) : o * W + 16 * s + frow);
    }
  };
  // element address of accumulator tile (o, s) at a uniform channel cu plus
  // the lane's channel cl in a [P][ld] bf16 tensor.  Whole-row tiles: the
  // pixel is a uniform part + the lane's part, so the address is a uniform
  // 64-bit base plus one 32-bit lane offset (the epilogue's 64-bit per-lane
  // addresses spilled next to the accumulators); row-segment tiles: the
  // pixel (out-of-image: pixel 0, never used)
  const int lpix = G::PAIR ? (frow >> 3) * 64 + (frow & 7) : frow;
  auto elem = [&](const void *base, int o, int s, int cu, int cl, int ld) __attribute__((always_inline))
      -> const char * {
    const char *b = reinterpret_cast<const char *>(base);
    if constexpr (G::SEGM) {
      long long p = pix_at(o, s);
      if (p < 0) p = 0;
      return b + (p * ld + cu + cl) * 2;
    } else {
      const long long up = (long long)p0 + wp * 128 + (G::PAIR ? o * 8 : o * W + 16 * s);
      return b + (up * ld + cu) * 2 + (uint32_t)(lpix * ld + cl) * 2u;
    }
  };
  // 16-B stores: per pair of 16-channel blocks (2p, 2p + 1) one
  // v_permlane16_swap per dword (odd rows of the first <-> even rows of the
  // second) leaves lane (row fq, pixel frow) with 8 consecutive channels at
  // 32 p + {0, 16, 8, 24}[fq]: 4 lanes write a pixel's 64 B (8-B stores of
  // 32-B pieces were store-issue bound)
  const int coff = (fq & 1) * 16 + (fq >> 1) * 8;
  auto swap_pair = [&](f32x4 &va, f32x4 &vb) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(va[j]), __float_as_uint(vb[j]),
                                                      false, false);
      va[j] = __uint_as_float(t[0]);
      vb[j] = __uint_as_float(t[1]);
    }
  };
  if constexpr (BNREG && ALLOW_BN) {
    if (a.bpart) {
      // ---- fused BN -> PReLU backward (rr_igemm_bnbwd; IgemmArgs::bpart)
      // in registers: the accumulator is dL/d(PReLU out); per lane 8
      // channels of one pixel per block pair.  The K loop's last barrier
      // freed the LDS: the channel constants go there ----
      float *cst = reinterpret_cast<float *>(smem);   // [4][BC] mean, invstd, aff_s, aff_b
      for (int i = tid; i < BC; i += G::NT) {
        cst[i] = a.bmean[c0 + i]; cst[BC + i] = a.binv[c0 + i];
        cst[2 * BC + i] = a.baff_s[c0 + i]; cst[3 * BC + i] = a.baff_b[c0 + i];
      }
      __syncthreads();
      const float al = a.balpha[0];
      // the wave tile's pre-BN inputs t first (every load in flight before
      // the first store, as in the register epilogue below)
      // (in two halves of the wave's rows, as the register epilogue's operand)
      constexpr int RHB = R / 2;
      uint4 tq[RHB * NS * (NM / 2)];
      auto preload_t = [&](int oh) __attribute__((always_inline)) {
#pragma unroll
        for (int o = oh; o < oh + RHB; ++o)
#pragma unroll
          for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int pp = 0; pp < NM / 2; ++pp)
              tq[((o - oh) * NS + s) * (NM / 2) + pp] =
                  *reinterpret_cast<const uint4 *>(elem(a.bt, o, s, c0 + cb + 32 * pp, coff, a.cout));
      };
      float g0[NM / 2][8], g1[NM / 2][8];
      double sa = 0.0;                                 // (fp64: igemm_epi.h store_staged_bnbwd)
#pragma unroll
      for (int pp = 0; pp < NM / 2; ++pp)
#pragma unroll
        for (int j = 0; j < 8; ++j) { g0[pp][j] = 0.f; g1[pp][j] = 0.f; }
#pragma unroll
      for (int o = 0; o < R; ++o) {
        if (o % RHB == 0) preload_t(o);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const long long p = pix_at(o, s);
#pragma unroll
          for (int pp = 0; pp < NM / 2; ++pp) {
            f32x4 va = acc[o][s][2 * pp], vb = acc[o][s][2 * pp + 1];
            swap_pair(va, vb);
            if (p < 0) continue;
            const int cl = cb + 32 * pp + coff;          // column in the block
            const uint4 tr = tq[((o % RHB) * NS + s) * (NM / 2) + pp];
            const f32x4 t0 = f32x4{__uint_as_float(tr.x << 16), __uint_as_float(tr.x & 0xffff0000u),
                                   __uint_as_float(tr.y << 16), __uint_as_float(tr.y & 0xffff0000u)};
            const f32x4 t1 = f32x4{__uint_as_float(tr.z << 16), __uint_as_float(tr.z & 0xffff0000u),
                                   __uint_as_float(tr.w << 16), __uint_as_float(tr.w & 0xffff0000u)};
            const float g[8] = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
            const float t[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
            float gm[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float u = t[j] * cst[2 * BC + cl + j] + cst[3 * BC + cl + j];   // BN out
              sa += u > 0.f ? 0.0 : (double)(g[j] * u);
              gm[j] = u > 0.f ? g[j] : al * g[j];
              g0[pp][j] += gm[j];
              g1[pp][j] += gm[j] * ((t[j] - cst[cl + j]) * cst[BC + cl + j]);
            }
            store8<bf16_t>(reinterpret_cast<bf16_t *>(const_cast<char *>(elem(a.y1, o, s, c0 + cb + 32 * pp, coff,
                                                                               a.cout))),
                           f32x4{gm[0], gm[1], gm[2], gm[3]}, f32x4{gm[4], gm[5], gm[6], gm[7]});
          }
        }
      }
      // over the 16 pixel lanes (row16_sum: the fixed xor-tree order), then one partial row per
      // wave row: [srow][cout][3] = (sum gm, sum gm * xhat, 0)
#pragma unroll
      for (int pp = 0; pp < NM / 2; ++pp)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          g0[pp][j] = row16_sum(g0[pp][j]);
          g1[pp][j] = row16_sum(g1[pp][j]);
        }
      if (frow == 0) {
#pragma unroll
        for (int pp = 0; pp < NM / 2; ++pp) {
          f32x4 *bp = reinterpret_cast<f32x4 *>(a.bpart + ((long long)srow * a.cout + c0 + cb + 32 * pp + coff) * 3);
          bp[0] = f32x4{g0[pp][0], g1[pp][0], 0.f, g0[pp][1]};
          bp[1] = f32x4{g1[pp][1], 0.f, g0[pp][2], g1[pp][2]};
          bp[2] = f32x4{0.f, g0[pp][3], g1[pp][3], 0.f};
          bp[3] = f32x4{g0[pp][4], g1[pp][4], 0.f, g0[pp][5]};
          bp[4] = f32x4{g1[pp][5], 0.f, g0[pp][6], g1[pp][6]};
          bp[5] = f32x4{0.f, g0[pp][7], g1[pp][7], 0.f};
        }
      }
      // the PReLU alpha partial: [srow][cout / 64], one value per 64
      // channels (a 32-channel wave adds its partner's through LDS)
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) sa += __shfl_xor(sa, off, 64);
      float *ap = a.bapart + (long long)srow * (a.cout / 64) + (c0 + cb) / 64;
      if constexpr (NW == 64) {
        if (lane == 0) *ap = (float)sa;
      } else {
        double *red = reinterpret_cast<double *>(cst + 4 * BC);
        if (lane == 0) red[wv] = sa;
        __syncthreads();
        if (lane == 0 && (wc & 1) == 0) *ap = (float)(sa + red[wv + 1]);
      }
      return;
    }
  }
  if constexpr (EPI == 3 && BNREG) return;           // (a.bpart: returned above)
  if (EPI != 3 && (BNREG || !ALLOW_BN || !a.bpart)) {
    // ---- register epilogue: lane = 4 NHWC channels of one pixel per
    // accumulator tile ----
    if (a.stats) {
      // per-channel partial sums of the pre-bias accumulator over the wave's
      // 128 pixels: over (o, s) in registers, then over the 16 pixel lanes
      // (row16_sum: the fixed xor-tree order), one partial row per 128 pixels
      f32x4 s1[NM], s2[NM];
#pragma unroll
      for (int m = 0; m < NM; ++m) { s1[m] = f32x4{0.f, 0.f, 0.f, 0.f}; s2[m] = s1[m]; }
#pragma unroll
      for (int o = 0; o < R; ++o)
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bool ok = !G::SEGM || pix_at(o, s) >= 0;
#pragma unroll
          for (int m = 0; m < NM; ++m) {
            const f32x4 v = ok ? acc[o][s][m] : f32x4{0.f, 0.f, 0.f, 0.f};
            s1[m] += v;
            s2[m] += v * v;
          }
        }
      // over the 16 pixel lanes by a reduce-scatter: V[k] = (s1, s2) of
      // (m, j) = divmod(k / 2, 4); each step pairs lanes that differ in one bit
      // of frow (row mirror: bit 3, half mirror: 2, xor 2: 1, xor 1: 0), the
      // lane with the bit clear keeps the lower half of its values plus its
      // partner's copy, the other the upper half: 8 NM - 2 adds instead of 32
      // NM (four-step tree per value).  Lane frow ends with V[NV/16 frow ..]
      constexpr int NV = 8 * NM;
      float v[NV];
#pragma unroll
      for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[(m * 4 + j) * 2] = s1[m][j]; v[(m * 4 + j) * 2 + 1] = s2[m][j]; }
      auto rs_step = [&](int n, bool hi, auto CTRLc) __attribute__((always_inline)) {
        constexpr int CTRL = decltype(CTRLc)::value;
#pragma unroll
        for (int i = 0; i < NV / 2; ++i) {
          if (i >= n / 2) break;
          const float send = hi ? v[i] : v[i + n / 2];
          const float keep = hi ? v[i + n / 2] : v[i];
          v[i] = keep + dpp_f<CTRL>(send);
        }
      };
      rs_step(NV, (frow & 8) != 0, ic<DPP_MIRROR>{});
      rs_step(NV / 2, (frow & 4) != 0, ic<DPP_HALF_MIRROR>{});
      rs_step(NV / 4, (frow & 2) != 0, ic<DPP_XOR2>{});
      rs_step(NV / 8, (frow & 1) != 0, ic<DPP_XOR1>{});
      float *sp = a.stats + ((long long)srow * a.cout + c0 + cb) * 2;
      if constexpr (NV / 16 == 2) {
        // (s1, s2) of (m, j) = divmod(frow, 4)
        const int ch = (frow >> 2) * 16 + fq * 4 + (frow & 3);
        *reinterpret_cast<float2 *>(sp + ch * 2) = make_float2(v[0], v[1]);
      } else {
        static_assert(NV / 16 == 1, "16- or 32-value reductions");
        // t = frow & 1 of (m, j) = divmod(frow / 2, 4)
        const int ch = (frow >> 3) * 16 + fq * 4 + ((frow >> 1) & 3);
        sp[ch * 2 + (frow & 1)] = v[0];
      }
    }
    f32x4 bv[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) bv[m] = *reinterpret_cast<const f32x4 *>(lbias + cb + m * 16 + fq * 4);
    const int ld1 = a.split > 0 ? a.split : a.cout;
    const int ld2 = a.cout - a.split;
    // rr_igemm_ex RR_ACT_POOL: the 2x2 max-pool of the activated output
    // (MaxPool2d(2, 2) after an encoder block / a VGG conv+ReLU, floor
    // sizes) to a.ypool [n][h/2][w/2][c_out]; RR_ACT_NOFULL: only that.
    // Rows are finished in pairs (o, o + 1: a wave's first row is even), the
    // column pair is lane frow ^ 1 (same 8 channels after the swap)
    const bool pool = ALLOW_POOL && (a.act & RR_ACT_POOL) != 0, full = !ALLOW_POOL || (a.act & RR_ACT_NOFULL) == 0;
    const int ph = a.h >> 1, pw = a.w >> 1;
    // one epilogue operand of the whole wave tile -- the accumulate input,
    // else the residual, else the ReLU mask (uniform) -- is loaded before the
    // first store: a store may alias a later load, so the compiler keeps them
    // in program order, and loaded next to its use every 16-B group paid a
    // memory latency of its own (the 32x32 dgrads ran 30-70 % over the plain
    // conv).  A second operand (accumulate AND mask) still loads in place.
    const int pre = (ALLOW_OPS && a.accumulate) ? 1 : ((ALLOW_EX && a.res) ? 2 : ((ALLOW_OPS && a.has_mask) ? 3 : 0));
    // operand / destination address of tile (o, s), block pair pp (the
    // concat split is uniform per pair: split % 32 == 0)
    auto op_ptr = [&](int kind, int o, int s, int pp) __attribute__((always_inline)) -> const char * {
      const int cu = c0 + cb + 32 * pp;
      if (kind == 1) {
        const bool second = a.split > 0 && cu >= a.split;
        return second ? elem(a.y2, o, s, cu - a.split, coff, ld2) : elem(a.y1, o, s, cu, coff, ld1);
      }
      return elem(kind == 2 ? a.res : a.mask, o, s, cu, coff, ld1);
    };
    // (in two halves of the wave's rows: the whole tile's operand, 64 VGPRs
    // on the 128 x 64 tiles, spilled next to the accumulators)
    constexpr int RH = R >= 4 ? R / 2 : R;            // rows per half (even: row pairs stay whole)
    constexpr int NQ = RH * NS * (NM / 2);
    uint4 opq[NQ];
    auto preload = [&](int oh) __attribute__((always_inline)) {
      if (!pre) return;
#pragma unroll
      for (int o = oh; o < oh + RH; ++o)
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int pp = 0; pp < NM / 2; ++pp)
            opq[((o - oh) * NS + s) * (NM / 2) + pp] =
                *reinterpret_cast<const uint4 *>(op_ptr(pre, o, s, pp));
    };
    static_assert(RH % 2 == 0, "halves of whole row pairs");
    auto unpack8 = [](const uint4 r, f32x4 &lo, f32x4 &hi) __attribute__((always_inline)) {
      lo = f32x4{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                 __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u)};
      hi = f32x4{__uint_as_float(r.z << 16), __uint_as_float(r.z & 0xffff0000u),
                 __uint_as_float(r.w << 16), __uint_as_float(r.w & 0xffff0000u)};
    };
#pragma unroll
    for (int o2 = 0; o2 < R; o2 += 2) {
      if (o2 % RH == 0) preload(o2);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
#pragma unroll
        for (int pp = 0; pp < NM / 2; ++pp) {
          f32x4 fin[2][2];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int o = o2 + t;
            const long long p = pix_at(o, s);
            f32x4 va = acc[o][s][2 * pp] + bv[2 * pp], vb = acc[o][s][2 * pp + 1] + bv[2 * pp + 1];
            swap_pair(va, vb);
            fin[t][0] = va;
            fin[t][1] = vb;
            if (G::SEGM && p < 0) continue;
            bf16_t *dst = reinterpret_cast<bf16_t *>(const_cast<char *>(op_ptr(1, o, s, pp)));
            const int q = ((o % RH) * NS + s) * (NM / 2) + pp;
            if (ALLOW_OPS && a.accumulate) {
              f32x4 lo, hi;
              unpack8(opq[q], lo, hi);                      // (pre == 1)
              va += lo;
              vb += hi;
            }
            if (ALLOW_EX && a.res) {                       // (rr_igemm_ex: y1's layout, no split)
              f32x4 lo, hi;
              if (pre == 2) {
                unpack8(opq[q], lo, hi);
              } else {
                const bf16_t *rp = reinterpret_cast<const bf16_t *>(op_ptr(2, o, s, pp));
                lo = load4<bf16_t>(rp);
                hi = load4<bf16_t>(rp + 4);
              }
              va += lo;
              vb += hi;
            }
            if ((a.act & 3) == RR_ACT_RELU) {
#pragma unroll
              for (int j = 0; j < 4; ++j) { va[j] = fmaxf(va[j], 0.f); vb[j] = fmaxf(vb[j], 0.f); }
            } else if (ALLOW_EX && (a.act & 3) == RR_ACT_PRELU) {
              const float al = a.alpha[0];
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                va[j] = va[j] > 0.f ? va[j] : al * va[j];
                vb[j] = vb[j] > 0.f ? vb[j] : al * vb[j];
              }
            }
            if (ALLOW_OPS && a.has_mask) {
              f32x4 ma, mb;
              if (pre == 3) {
                unpack8(opq[q], ma, mb);
              } else {
                const bf16_t *mp = reinterpret_cast<const bf16_t *>(op_ptr(3, o, s, pp));
                ma = load4<bf16_t>(mp);
                mb = load4<bf16_t>(mp + 4);
              }
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                va[j] = ma[j] > 0.f ? va[j] : 0.f;
                vb[j] = mb[j] > 0.f ? vb[j] : 0.f;
              }
            }
            fin[t][0] = va;
            fin[t][1] = vb;
            if (full) store8<bf16_t>(dst, va, vb);
          }
          if (pool) {
            // the window in window order -- (o2, x) own, (o2, x + 1) the xor-1
            // lane's, (o2 + 1, x) own, (o2 + 1, x + 1) the neighbour's -- on the
            // bf16-rounded values (the stored ones maxpool_fwd8 reads): the
            // first max and its index (rr_igemm_pool's a.pidx)
            f32x4 m0, m1;
            uint32_t id[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float u0 = bf16_to_f32(f32_to_bf16(fin[0][j >> 2][j & 3]));
              const float u1 = bf16_to_f32(f32_to_bf16(fin[1][j >> 2][j & 3]));
              const float v0 = __uint_as_float(xor1_u32(__float_as_uint(u0)));
              const float v1 = __uint_as_float(xor1_u32(__float_as_uint(u1)));
              const float m = pool4_first_max(u0, v0, u1, v1, id[j]);
              if (j < 4) m0[j] = m;
              else m1[j - 4] = m;
            }
            const long long p = pix_at(o2, s);            // the window's top-left pixel
            if ((frow & 1) == 0 && (!G::SEGM || p >= 0)) {
              const int n = (int)(p / ((long long)a.h * a.w));
              const int rem = (int)(p - (long long)n * a.h * a.w);
              const int y = rem / a.w, x = rem - (rem / a.w) * a.w;
              if (y + 1 < a.h && x + 1 < a.w) {             // (floor: a last odd row / column drops)
                const int c = c0 + cb + 32 * pp + coff;
                const long long q = (((long long)n * ph + (y >> 1)) * pw + (x >> 1)) * a.cout + c;
                store8<bf16_t>(reinterpret_cast<bf16_t *>(a.ypool) + q, m0, m1);
                if (a.pidx)
                  *reinterpret_cast<uint2 *>(a.pidx + q) =
                      make_uint2(id[0] | (id[1] << 8) | (id[2] << 16) | (id[3] << 24),
                                 id[4] | (id[5] << 8) | (id[6] << 16) | (id[7] << 24));
              }
            }
          }
        }
      }
    }
    return;
  }
  if constexpr (!BNREG && ALLOW_BN) {
    // ---- BN-backward epilogue: one 128-pixel group (= one wave row of the
    // grid) at a time as fp32 [128][BC] in LDS, then the staged store ----
    float *stg = reinterpret_cast<float *>(smem);
    for (int g = 0; g < G::WP; ++g) {
      if (wp == g) {
#pragma unroll
        for (int o = 0; o < R; ++o)
#pragma unroll
          for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int m = 0; m < NM; ++m) {
              const int r = G::PAIR ? (frow >> 3) * 64 + o * 8 + (frow & 7) : o * W + 16 * s + frow;
              const int col = wc * NW + m * 16 + fq * 4;
              *reinterpret_cast<f32x4 *>(stg + r * G::SROW + col) = acc[o][s][m];
            }
      }
      __syncthreads();
      store_staged<bf16_t, BC, 128, G::NT, RR_CONV3X3>(a, stg, c0, p0 + g * 128, p0 / 128 + g, tid);
      __syncthreads();
    }
  }
}

// column block and per-wave channels for *d: BC = 128 / 64 by c_out, 128 x
// 64 wave tiles, except where that leaves fewer than 256 workgroups (one per
// CU): the 8x8 256-channel layers (B = 512: 128 tiles) take 128 x 32 wave
// tiles.  sg > 0: row-segment tiles (any H x W)
struct R3Pick { int bc, nw, nwv, hb, sg; };
int r3_tpx(R3Pick k) { return (k.nwv / (k.bc / k.nw)) * 128; }

// square 8 / 16 / 32 / 64 maps whose pixel count fills whole tiles take the
// whole-row tiles; everything else (the reference's 224 / 112 / 56 / 28 /
// 14 maps, odd sizes, small batches) the row-segment tiles: 32-column
// segments x 4 rows per wave above W = 16, 16 x 8 at W <= 16.
// Workgroups of whole-row tiles: one 8-wave workgroup per CU with a
// double-buffered halo where c_out % 128 == 0 on the 16x16 / 8x8 maps
// (5-12% faster there, profiles/r3i_ab.jsonl, r4z_conv3r_wg_ab.jsonl), else
// 4-wave workgroups, 2 per CU (one's epilogue / DMA waits overlap the other's
// MFMAs) with one halo buffer -- also at W = 32, where the 8-wave tiles were
// 4-11 % slower once the row loop lost its run-time switches (r4z).  The
// 128-channel column blocks are 2-3 % faster per layer than 256-channel ones
// at 16x16 / 8x8 (profiles/r4zk_conv3r_bc_ab.jsonl).  Test overrides
// (RR_PATH, common.h): conv3r_wg=4 / 8 forces a workgroup kind,
// conv3r_w64=0 puts the 64x64 maps on row-segment tiles, conv3r_segwg=4 / 8
// the row-segment workgroup kind
R3Pick r3_pick(const rr_igemm_desc *d) {
  const long long P = (long long)d->n * d->h * d->w;
  const int W = d->w;
  const bool w64 = W == 64 && rr_path("conv3r_w64", 1) != 0;
  const bool square = d->h == W && (W == 8 || W == 16 || W == 32 || w64);
  const int fwg = rr_path("conv3r_wg", 0);
  const int nwv = fwg == 4 || fwg == 8 ? fwg : (d->c_out % 128 == 0 && W != 32 ? 8 : 4);
  if (square) {
    R3Pick c[3];
    int nc = 0;
    if (nwv == 8) {
      if (d->c_out % 256 == 0 && W == 8 && (P / 256) * (d->c_out / 256) < 256 && P % 256 == 0) {
        c[nc++] = {128, 32, 8, 2, 0};
      } else if (d->c_out % 128 == 0) {
        c[nc++] = {128, 64, 8, 2, 0};
      } else {
        c[nc++] = {64, 32, 8, 2, 0};
      }
    } else if (d->c_out % 128 == 0) {
      // 128-channel column blocks of 128 x 64 wave tiles (256-pixel tiles);
      // below 512 workgroups (2 per CU) the 8x8 layers take 128 x 32 wave
      // tiles (128-pixel tiles)
      if (W == 8 && (P / 256) * (d->c_out / 128) < 512 && P % 128 == 0) c[nc++] = {128, 32, 4, 1, 0};
      else c[nc++] = {128, 64, 4, 1, 0};
    } else {
      c[nc++] = {64, 64, 4, 1, 0};
    }
    // batches whose pixels do not fill the first pick's tiles: smaller
    // whole-row tiles before the row-segment ones (an odd batch of 16x16
    // 256-channel maps stays on whole rows)
    if (d->c_out % 128 == 0) {
      c[nc++] = {128, 32, 8, 2, 0};
      c[nc++] = {128, 32, 4, 1, 0};
    } else {
      c[nc++] = {64, 32, 4, 1, 0};
    }
    for (int i = 0; i < nc; ++i)
      if (P % r3_tpx(c[i]) == 0) return c[i];
  }
  const int sg = W > 16 ? 2 : 1;
  // one 8-wave workgroup per CU with a double-buffered halo (the next
  // chunk loads during this one's stages) on the 128+-channel maps of
  // W <= 28 (the 28x28 / 14x14 layers: 9-12 % faster), 2 x 4-wave elsewhere
  // (the 224 / 112 / 56 layers: even or 5-10 % slower,
  // profiles/r3v_ab224_segwg.jsonl)
  const int fsw = rr_path("conv3r_segwg", 0);
  const int segwg = fsw == 4 || fsw == 8 ? fsw : (d->c_out % 128 == 0 && W <= 28 ? 8 : 4);
  if (segwg == 8) {
    if (sg == 2) return d->c_out % 128 == 0 ? R3Pick{128, 64, 8, 2, 2} : R3Pick{64, 32, 8, 2, 2};
    return d->c_out % 128 == 0 ? R3Pick{128, 32, 8, 2, 1} : R3Pick{64, 32, 8, 1, 1};
  }
  if (sg == 2) return d->c_out % 128 == 0 ? R3Pick{128, 64, 4, 1, 2} : R3Pick{64, 64, 4, 1, 2};
  return d->c_out % 128 == 0 ? R3Pick{128, 32, 4, 1, 1} : R3Pick{64, 32, 4, 1, 1};
}
// row-segment tiles: rows per tile, column segments and row bands per image
int r3_tr(R3Pick k) { return (k.nwv / (k.bc / k.nw)) * (8 / k.sg); }
long long r3_seg_tiles(const rr_igemm_desc *d, R3Pick k) {
  const long long nseg = (d->w + 16 * k.sg - 1) / (16 * k.sg), nband = (d->h + r3_tr(k) - 1) / r3_tr(k);
  return (long long)d->n * nseg * nband;
}
// pixel tiles of the launch
long long r3_ptiles(const rr_igemm_desc *d, R3Pick k) {
  if (k.sg) return r3_seg_tiles(d, k);
  return (long long)d->n * d->h * d->w / r3_tpx(k);
}

}  // namespace

// RR_PATH conv3r=0: the halo / tiled kernels instead (tests), conv3r=2:
// whole-row tiles only
int conv3r_bc(const rr_igemm_desc *d) {
  const int mode = rr_path("conv3r", 1);
  if (mode == 0) return 0;
  if (!d || d->dtype != RR_BF16 || d->mode != RR_CONV3X3 || d->out_nchw) return 0;
  if (d->n <= 0 || d->h <= 0 || d->w <= 0) return 0;
  if (d->c_in1 <= 0 || d->c_in1 % 32 || d->c_in2 % 32 || d->c_out % 64) return 0;
  if (d->out_split && (d->out_split % 32 || d->out_split >= d->c_out)) return 0;
  const R3Pick k = r3_pick(d);
  if (k.sg && mode == 2) return 0;
  const long long tiles = r3_ptiles(d, k) * (d->c_out / k.bc);
  if (tiles <= 0 || tiles > 0x7fffffffLL) return 0;
  return k.bc;
}

int conv3r_stat_blocks(const rr_igemm_desc *d) {
  if (!conv3r_bc(d)) return 0;
  const R3Pick k = r3_pick(d);
  return (int)(r3_ptiles(d, k) * (k.nwv / (k.bc / k.nw)));   // one row per wave row of a tile
}

// the specialised epilogue instances wherever the call allows one: EPI 1
// (plain: bias / statistics / ReLU / split, no operand loads) for the
// training step's forward and plain dgrads, 4 (+ pool), 3 (the fused BN
// backward alone), 2 (+ accumulate / ReLU-mask operands); the general one
// (0) otherwise
template <int W_, int BC, int NW, int NWV, int HB, int SG>
static void c3_launch(const IgemmArgs &a, dim3 grid, dim3 block, hipStream_t st) {
  const bool plain = !a.accumulate && !a.res && !a.has_mask && (a.act & 3) != RR_ACT_PRELU &&
                     !(a.act & (RR_ACT_POOL | RR_ACT_NOFULL)) && !a.bpart;
  if (plain) {
    hipLaunchKernelGGL((conv3r_kernel<W_, BC, NW, NWV, HB, SG, 1>), grid, block, 0, st, a);
    return;
  }
  const bool ex = a.res || (a.act & 3) == RR_ACT_PRELU || (a.act & (RR_ACT_POOL | RR_ACT_NOFULL));
  if ((a.act & RR_ACT_POOL) && !a.res && (a.act & 3) != RR_ACT_PRELU && !a.accumulate && !a.has_mask &&
      !a.bpart) {
    hipLaunchKernelGGL((conv3r_kernel<W_, BC, NW, NWV, HB, SG, 4>), grid, block, 0, st, a);
    return;
  }
  if (a.bpart && !ex && !a.accumulate && !a.has_mask) {
    hipLaunchKernelGGL((conv3r_kernel<W_, BC, NW, NWV, HB, SG, 3>), grid, block, 0, st, a);
    return;
  }
  if (!a.bpart && !ex) {
    hipLaunchKernelGGL((conv3r_kernel<W_, BC, NW, NWV, HB, SG, 2>), grid, block, 0, st, a);
    return;
  }
  if (!a.bpart && !a.accumulate && !a.has_mask) {
    hipLaunchKernelGGL((conv3r_kernel<W_, BC, NW, NWV, HB, SG, 5>), grid, block, 0, st, a);
    return;
  }
  hipLaunchKernelGGL((conv3r_kernel<W_, BC, NW, NWV, HB, SG, 0>), grid, block, 0, st, a);
}

template <int BC, int NW, int NWV, int HB, int SG>
static int conv3r_go(const rr_igemm_desc *d, IgemmArgs &a, hipStream_t st) {
  a.ncblk = a.cout / BC;
  const long long nblk = r3_ptiles(d, R3Pick{BC, NW, NWV, HB, SG}) * a.ncblk;
  if (nblk <= 0 || nblk > 0x7fffffffLL) return RR_EUNSUPPORTED;
  const dim3 grid((unsigned)nblk), block(64 * NWV);
  if constexpr (SG > 0) {
    c3_launch<0, BC, NW, NWV, HB, SG>(a, grid, block, st);
  } else {
    switch (d->w) {
      case 64: c3_launch<64, BC, NW, NWV, HB, 0>(a, grid, block, st); break;
      case 32: c3_launch<32, BC, NW, NWV, HB, 0>(a, grid, block, st); break;
      case 16: c3_launch<16, BC, NW, NWV, HB, 0>(a, grid, block, st); break;
      default: c3_launch<8, BC, NW, NWV, HB, 0>(a, grid, block, st); break;
    }
  }
  RR_CHECK_LAUNCH();
  return RR_OK;
}

int conv3r_launch(const rr_igemm_desc *d, IgemmArgs &a, hipStream_t st) {
  if (!conv3r_bc(d)) return RR_EUNSUPPORTED;
  const R3Pick k = r3_pick(d);
  if (k.sg == 2) {
    if (k.nwv == 8) {
      if (k.bc == 128) return conv3r_go<128, 64, 8, 2, 2>(d, a, st);
      return conv3r_go<64, 32, 8, 2, 2>(d, a, st);
    }
    if (k.bc == 128) return conv3r_go<128, 64, 4, 1, 2>(d, a, st);
    return conv3r_go<64, 64, 4, 1, 2>(d, a, st);
  }
  if (k.sg == 1) {
    if (k.nwv == 8) {
      if (k.bc == 128) return conv3r_go<128, 32, 8, 2, 1>(d, a, st);
      return conv3r_go<64, 32, 8, 1, 1>(d, a, st);
    }
    if (k.bc == 128) return conv3r_go<128, 32, 4, 1, 1>(d, a, st);
    return conv3r_go<64, 32, 4, 1, 1>(d, a, st);
  }
  if (k.nwv == 8) {
    if (k.bc == 128 && k.nw == 64) return conv3r_go<128, 64, 8, 2, 0>(d, a, st);
    if (k.bc == 128) return conv3r_go<128, 32, 8, 2, 0>(d, a, st);
    return conv3r_go<64, 32, 8, 2, 0>(d, a, st);
  }
  if (k.bc == 128 && k.nw == 64) return conv3r_go<128, 64, 4, 1, 0>(d, a, st);
  if (k.bc == 128) return conv3r_go<128, 32, 4, 1, 0>(d, a, st);
  if (k.nw == 64) return conv3r_go<64, 64, 4, 1, 0>(d, a, st);
  return conv3r_go<64, 32, 4, 1, 0>(d, a, st);
}

const char *conv3r_name(const rr_igemm_desc *d) {
  if (!conv3r_bc(d)) return "invalid";
  const R3Pick k = r3_pick(d);
  static char names[4][5][2][40];
  static char segnames[2][2][2][40];
  char *n;
  if (k.sg) {
    // conv3r_kernel<s2,BC> (32-column segments), <s1,BC> (16-column); ",w8":
    // 8-wave workgroups
    n = segnames[k.sg - 1][k.bc == 128][k.nwv == 8];
    if (!n[0]) snprintf(n, 40, "conv3r_kernel<s%d,%d%s>", k.sg, k.bc, k.nwv == 8 ? ",w8" : "");
    return n;
  }
  const int wi = d->w == 8 ? 0 : d->w == 16 ? 1 : d->w == 32 ? 2 : 3;
  const int bi = k.bc == 64 ? (k.nw == 64 ? 0 : 4) : (k.nw == 64 ? 1 : 2);
  const int vi = k.nwv == 8;
  n = names[wi][bi][vi];
  if (!n[0]) {
    // conv3r_kernel<W,BC> (128 x 64 wave tiles), <W,BC,32> (128 x 32); the
    // 8-wave one-per-CU variant adds ",w8"
    snprintf(n, 40, "conv3r_kernel<%d,%d%s%s>", d->w, k.bc, k.nw == 32 ? ",32" : "", vi ? ",w8" : "");
  }
  return n;
}

#ifdef RR_CONV3R_STAMPS
extern "C" int rr_conv3r_stamps(unsigned long long *host, int n, int clear) {
  if (n > (1 << 18)) n = 1 << 18;
  if (host && hipMemcpyFromSymbol(host, HIP_SYMBOL(rr_c3_stamps), (size_t)n * 8) != hipSuccess) return -3;
  if (clear) {
    static unsigned long long z[1 << 18];
    if (hipMemcpyToSymbol(HIP_SYMBOL(rr_c3_stamps), z, sizeof(z)) != hipSuccess) return -3;
  }
  return 0;
}
#endif
