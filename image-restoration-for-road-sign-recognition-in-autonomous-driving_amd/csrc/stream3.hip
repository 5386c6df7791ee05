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
//     output rows (whole images at batch 512) in 128-pixel steps
//     (RPS = 128 / W rows);
//   * every input row is read ONCE: rows land by LDS-DMA
//     (global_load_lds_dwordx4) in a ring of RING padded rows, D steps ahead
//     of the MFMAs; a step's three input-row windows for the taps are slots
//     of that ring (the zero padding rows / columns come from a zero page);
//   * the weights (64 x 576 bf16 = 72 KB) live in registers for the whole
//     kernel: wave (wc, wp) owns output channels [32 wc, 32 wc + 32) -- its
//     A fragments, 144 VGPRs -- and 32 pixels of each step;
//   * the epilogue stores from the accumulators (4 NHWC channels per lane)
//     and keeps BN statistics / BN-backward sums in registers across all the
//     workgroup's steps (one reduction at the end, per-workgroup partials).
//
// Ring row image ("k-planes", as the halo kernel): plane j = 16-B channel
// chunk j of the W + 2 padded pixels, plane size PL = 0 mod 256 B, so a
// ds_read_b128 16-lane group (8 pixels of chunk q, 8 of chunk q + 1 --
// the MFMA B fragment map) hits 16 distinct bank slots for any pixel base.
//
// vmcnt accounting: LDS-DMA, the epilogue's global loads and its stores share
// the in-order vector-memory counter.  Iteration u issues, in this order:
// epilogue loads E(u), DMA(u + D) (DMAW per wave), stores S(u).  Before step
// v reads the ring, a wave waits until at most
//   (D - 1) DMAW + S [v-D computed] + (E + S) * #computed in (v-D, v)
// of its ops are outstanding (exactly the ops younger than DMA(v)), then a
// raw s_barrier publishes every wave's rows.  A plain __syncthreads would
// drain all DMA in flight (vmcnt(0)).
#include "common.h"
#include "stream3.h"

#include <climits>
#include <cstdlib>

namespace {

constexpr int S3_WG = 256;   // workgroups: one per CU on MI355X (fixed: deterministic partial rows)

template <int W> struct S3Geo {
  static constexpr int RPS = 128 / W;                          // image rows per step
  static constexpr int PL = W == 64 ? 1536 : 768;              // plane bytes >= (W + 2) * 16
  static constexpr int ROWB = 8 * PL;                          // one padded row, 64 channels
  static constexpr int SCRATCH = 4096;                         // bnbwd coefficients
  static constexpr int RING = (((160 * 1024 - SCRATCH) / ROWB) / RPS) * RPS;
  static constexpr int D = (RING - 2) / RPS - 1;               // steps of prefetch in flight
  static constexpr int DMAW = RPS * ROWB / 1024 / 8;           // DMA instructions / wave / step
  static constexpr int LDS = RING * ROWB + SCRATCH;
  static_assert((RPS * ROWB) % 8192 == 0, "a step's rows must split evenly over 8 waves");
  static_assert(PL % 256 == 0 && PL >= (W + 2) * 16, "plane size");
  static_assert(D >= 2 && (D + 1) * RPS + 2 <= RING, "ring");
};

enum { S3_PRE = 0, S3_COMP = 1 };
enum { EPI_PLAIN = 0, EPI_LOAD = 1, EPI_BNBWD = 2 };

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

typedef unsigned long long u64;

// 8-byte global load the compiler's waitcnt pass does not see (the caller
// waits with an explicit vmcnt that names the result registers)
__device__ __forceinline__ u64 load_b64_async(const char *p) {
  u64 r;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
// LDS read of 8 bytes outside the compiler's view: its waitcnt pass puts a
// vmcnt(0) (drain all LDS-DMA) before a visible ds_read it cannot separate
// from the DMA destination
__device__ __forceinline__ void lds_read_2x4(const float *p, f32x4 &lo, f32x4 &hi) {
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(lo), "=v"(hi) : "v"(a) : "memory");
}
__device__ __forceinline__ f32x4 unpack4(u64 v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  return f32x4{__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
               __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
}

struct Cur {
  int kind, n, y0, c;   // virtual step: pre-load or compute of output rows [y0, y0 + RPS) of image n
};

template <int W, int EPI>
__global__ __launch_bounds__(512, 2) void stream3_kernel(S3Args a, int nsteps) {
  using G = S3Geo<W>;
  constexpr int RPS = G::RPS, PL = G::PL, ROWB = G::ROWB, RING = G::RING, D = G::D;
  constexpr int DMAW = G::DMAW;
  constexpr int MC = 2, MP = 2;                 // 32 channels x 32 pixels per wave
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  float *coef = reinterpret_cast<float *>(smem + RING * ROWB);   // [64][2]

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wc = wv & 1, wp = wv >> 1;
  const int frow = lane & 15, fq = lane >> 4;
  const int H = a.h;
  const int spi = H / RPS;                      // compute steps per image
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
            *reinterpret_cast<const bf16x8 *>(a.wt + ((co * 9 + tap) * 64 + kb * 32 + fq * 8) * 2);
  }
  f32x4 bia[MC];
#pragma unroll
  for (int mi = 0; mi < MC; ++mi) {
    const int c = wc * 32 + mi * 16 + fq * 4;
    bia[mi] = a.bias ? *reinterpret_cast<const f32x4 *>(a.bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float al = 0.f;
  if constexpr (EPI == EPI_BNBWD) {
    if (tid < 64) {
      // u = t * s + b (BN out = PReLU in)
      coef[tid * 2 + 0] = a.baff_s[tid];
      coef[tid * 2 + 1] = a.baff_b[tid];
    }
    al = a.balpha[0];
    __syncthreads();
  }

  // ---- LDS-DMA lanes: row-in-step and byte offset inside a pixel row --------
  const long long zoff = (long long)((uintptr_t)rr_zero_page - (uintptr_t)a.x);   // zero rows
  int drow[DMAW], dofs[DMAW];
#pragma unroll
  for (int i = 0; i < DMAW; ++i) {
    const int off = (wv * DMAW + i) * 1024 + lane * 16;
    const int r = off / ROWB, o = off - r * ROWB;
    const int pl = o / PL, x = (o - pl * PL) / 16 - 1;
    drow[i] = r;
    dofs[i] = (x >= 0 && x < W) ? (x * 64 + pl * 8) * 2 : -1;
  }
  auto issue = [&](int v, const Cur &cu, bool live) __attribute__((always_inline)) {
    char *reg = smem + ((v * RPS) % RING) * ROWB;
#pragma unroll
    for (int i = 0; i < DMAW; ++i) {
      // keeps the compiler from hoisting DMAW 64-bit row bases out of the
      // loop (VGPR pressure: the weights hold 144)
      asm volatile("" : "+v"(dofs[i]));
      const int r = drow[i];
      int y = cu.kind == S3_PRE ? cu.y0 - RPS + 1 + r : cu.y0 + 1 + r;
      const bool ok = live && dofs[i] >= 0 && y >= 0 && y < H && (cu.kind != S3_PRE || r >= RPS - 2);
      // one base pointer + a selected offset: a pointer select (or one
      // across address spaces) becomes a divergent branch, i.e. two
      // exec-masked DMA instructions, which breaks the vmcnt accounting
      const long long off = ok ? ((long long)(cu.n * H + y) * W) * 128 + dofs[i] : zoff;
      __builtin_amdgcn_global_load_lds((const void *)(a.x + off),
                                       LDS_PTR(reg + (wv * DMAW + i) * 1024), 16, 0, 0);
    }
  };
  auto advance = [&](Cur &cu) __attribute__((always_inline)) {
    if (cu.kind == S3_PRE) {
      cu.kind = S3_COMP;
    } else {
      ++cu.c;
      cu.y0 += RPS;
      if (cu.y0 == H) { cu.y0 = 0; ++cu.n; cu.kind = S3_PRE; }
    }
  };

  // ---- per-wave pixel blocks of a step ----
  int bq[MP], bx[MP], lpart[MP];
#pragma unroll
  for (int ni = 0; ni < MP; ++ni) {
    const int p = wp * 32 + ni * 16;
    bq[ni] = p / W;
    bx[ni] = p % W;
    lpart[ni] = fq * PL + (bx[ni] + frow) * 16;
  }

  // running epilogue sums: stats (sum, sum sq) or bnbwd (sum gm, sum gm xhat)
  f32x4 r0[MC], r1[MC];
  float ra = 0.f;
#pragma unroll
  for (int mi = 0; mi < MC; ++mi) { r0[mi] = f32x4{0.f, 0.f, 0.f, 0.f}; r1[mi] = r0[mi]; }

  const int E = EPI == EPI_PLAIN ? 0
                                 : (EPI == EPI_BNBWD ? MC * MP
                                                     : MC * MP * ((a.accumulate ? 1 : 0) + (a.mask ? 1 : 0)));
  constexpr int S = MC * MP;

  // weights / bias / coefficients resident before any DMA is in flight: the
  // compiler's own wait for them would otherwise drain the prologue DMAs
  __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0) (gfx9 encoding)
  Cur ld, cp;
  ld.c = cbeg;
  ld.n = cbeg / spi;
  ld.y0 = (cbeg - ld.n * spi) * RPS;
  ld.kind = S3_PRE;
  cp = ld;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    issue(k, ld, ld.c < cend);
    advance(ld);
  }
  unsigned hist = 0;                            // bit j: iteration v-1-j computed
#pragma unroll 1
  for (int v = 0; cp.c < cend; ++v) {
    const int younger = (D - 1) * DMAW + (((hist >> (D - 1)) & 1) ? S : 0) +
                        (E + S) * __builtin_popcount(hist & ((1u << (D - 1)) - 1));
    wait_vm_barrier(younger);
    const bool comp = cp.kind == S3_COMP;
    const long long pix0 = (long long)(cp.n * H + cp.y0) * W;
    // epilogue loads BEFORE this iteration's DMA: the compiler's wait for
    // them then leaves the new DMA in flight (see the vmcnt accounting above)
    // (inline asm: with an LDS-DMA in flight hipcc waits vmcnt(0) for any
    // ordinary load's result, which would drain the prefetch every step)
    u64 ev0[MC][MP], ev1[MC][MP];
    if constexpr (EPI != EPI_PLAIN) {
      if (comp) {
#pragma unroll
        for (int mi = 0; mi < MC; ++mi)
#pragma unroll
          for (int ni = 0; ni < MP; ++ni) {
            const long long e = (pix0 + bq[ni] * W + bx[ni] + frow) * 64 + wc * 32 + mi * 16 + fq * 4;
            if constexpr (EPI == EPI_BNBWD) {
              ev0[mi][ni] = load_b64_async(a.bt + e * 2);
            } else {
              if (a.accumulate) ev0[mi][ni] = load_b64_async(a.y + e * 2);
              if (a.mask) ev1[mi][ni] = load_b64_async(a.mask + e * 2);
            }
          }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    issue(v + D, ld, ld.c < cend);
    advance(ld);
    if (comp) {
      f32x4 acc[MC][MP];
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int ni = 0; ni < MP; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int s0 = v * RPS - 2;               // ring slot of input row y0 - 1
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const char *rb[MP];
#pragma unroll
        for (int ni = 0; ni < MP; ++ni) rb[ni] = smem + ((s0 + bq[ni] + dy) % RING) * ROWB + lpart[ni];
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
            bf16x8 fb[MP];
#pragma unroll
            for (int ni = 0; ni < MP; ++ni)
              fb[ni] = *reinterpret_cast<const bf16x8 *>(rb[ni] + kb * 4 * PL + dx * 16);
#pragma unroll
            for (int mi = 0; mi < MC; ++mi)
#pragma unroll
              for (int ni = 0; ni < MP; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mi][dy * 3 + dx][kb], fb[ni],
                                                                     acc[mi][ni], 0, 0, 0);
          }
      }
      // ---- epilogue: lane = pixel (frow) x 4 channels ----
      if constexpr (EPI != EPI_PLAIN) {
        // the epilogue loads are older than this step's DMAW DMAs
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(%8)"
                     : "+v"(ev0[0][0]), "+v"(ev0[0][1]), "+v"(ev0[1][0]), "+v"(ev0[1][1]),
                       "+v"(ev1[0][0]), "+v"(ev1[0][1]), "+v"(ev1[1][0]), "+v"(ev1[1][1])
                     : "n"(DMAW));
      }
#pragma unroll
      for (int mi = 0; mi < MC; ++mi) {
        const int c = wc * 32 + mi * 16 + fq * 4;
        f32x4 k01, k23;                         // (s, b) of channels c .. c + 3
        if constexpr (EPI == EPI_BNBWD) lds_read_2x4(coef + c * 2, k01, k23);
#pragma unroll
        for (int ni = 0; ni < MP; ++ni) {
          const long long e = (pix0 + bq[ni] * W + bx[ni] + frow) * 64 + c;
          f32x4 g = acc[mi][ni];
          if constexpr (EPI == EPI_BNBWD) {
            const f32x4 t = unpack4(ev0[mi][ni]);
            f32x4 gm;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              // sum gm * xhat = inv (sum gm t) - inv mean (sum gm): the
              // affine part is applied once per channel at the end
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
            if (a.stats) {
              r0[mi] += g;
              r1[mi] += g * g;
            }
            g += bia[mi];
            if constexpr (EPI == EPI_LOAD) {
              if (a.accumulate) g += unpack4(ev0[mi][ni]);
            }
            if (a.act == RR_ACT_RELU) {
#pragma unroll
              for (int j = 0; j < 4; ++j) g[j] = fmaxf(g[j], 0.f);
            }
            if constexpr (EPI == EPI_LOAD) {
              if (a.mask) {
                const f32x4 mk = unpack4(ev1[mi][ni]);
#pragma unroll
                for (int j = 0; j < 4; ++j) g[j] = mk[j] > 0.f ? g[j] : 0.f;
              }
            }
          }
          uint2 o;
          o.x = (uint32_t)f32_to_bf16(g[0]) | ((uint32_t)f32_to_bf16(g[1]) << 16);
          o.y = (uint32_t)f32_to_bf16(g[2]) | ((uint32_t)f32_to_bf16(g[3]) << 16);
          *reinterpret_cast<uint2 *>(a.y + e * 2) = o;
        }
      }
    }
    hist = (hist << 1) | (comp ? 1u : 0u);
    advance(cp);
  }
  // drain the ring's trailing (dummy) DMA before the LDS is reused / released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- per-workgroup partials: lanes of one channel (frow) -> waves (wp) ----
  const bool want = EPI == EPI_BNBWD || a.stats;
  if (!want) return;
#pragma unroll
  for (int mi = 0; mi < MC; ++mi)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        r0[mi][j] += __shfl_xor(r0[mi][j], o, 64);
        r1[mi][j] += __shfl_xor(r1[mi][j], o, 64);
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
  if constexpr (EPI == EPI_BNBWD) {
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
    if constexpr (EPI == EPI_BNBWD) {
      float *pp = a.bpart + ((long long)blockIdx.x * 64 + tid) * 3;
      pp[0] = x;
      pp[1] = a.binv[tid] * (y - a.bmean[tid] * x);
      pp[2] = 0.f;
    } else {
      a.stats[((long long)blockIdx.x * 64 + tid) * 2 + 0] = x;
      a.stats[((long long)blockIdx.x * 64 + tid) * 2 + 1] = y;
    }
  }
  if constexpr (EPI == EPI_BNBWD) {
    if (tid == 0) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) s += red[4 * 64 * 2 + q];
      a.bapart[blockIdx.x] = s;
    }
  }
}

template <int W>
int launch_w(const S3Args &a, int nsteps, hipStream_t st) {
  const dim3 grid(S3_WG), block(512);
  if (a.bt) {
    hipLaunchKernelGGL((stream3_kernel<W, EPI_BNBWD>), grid, block, 0, st, a, nsteps);
  } else if (a.accumulate || a.mask) {
    hipLaunchKernelGGL((stream3_kernel<W, EPI_LOAD>), grid, block, 0, st, a, nsteps);
  } else {
    hipLaunchKernelGGL((stream3_kernel<W, EPI_PLAIN>), grid, block, 0, st, a, nsteps);
  }
  RR_CHECK_LAUNCH();
  return RR_OK;
}

}  // namespace

int stream3_blocks(const rr_igemm_desc *d) {
  const char *e = getenv("RR_STREAM3");
  if (e && !atoi(e)) return 0;
  if (d->dtype != RR_BF16 || d->mode != RR_CONV3X3) return 0;
  if (d->c_in1 != 64 || d->c_in2 != 0 || d->c_out != 64 || d->out_split || d->out_nchw) return 0;
  if (d->w != 64 && d->w != 32) return 0;
  const int rps = 128 / d->w;
  if (d->h % rps) return 0;
  const long long nsteps = (long long)d->n * d->h / rps;
  if (nsteps < S3_WG) return 0;                 // every workgroup gets >= 1 step
  if ((long long)d->n * d->h * d->w * 64 > INT_MAX) return 0;
  return S3_WG;
}

int stream3_launch(const rr_igemm_desc *d, const S3Args &a, hipStream_t st) {
  if (!stream3_blocks(d)) return RR_EUNSUPPORTED;
  const int nsteps = (int)((long long)d->n * d->h / (128 / d->w));
  if (d->w == 64) return launch_w<64>(a, nsteps, st);
  return launch_w<32>(a, nsteps, st);
}
