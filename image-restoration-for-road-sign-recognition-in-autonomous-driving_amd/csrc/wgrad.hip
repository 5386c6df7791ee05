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
};

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
  int bid = blockIdx.x;
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

  // partial[split][a][tap][b]
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
  long long want = (1024 + tiles - 1) / tiles;                  // ~1024 workgroups
  long long maxs = (P + 4 * BKP_PLAN - 1) / (4 * BKP_PLAN);     // >= 4 stages per split
  long long ns = want < maxs ? want : maxs;
  if (ns < 1) ns = 1;
  long long len = (P + ns - 1) / ns;
  len = (len + BKP_PLAN - 1) / BKP_PLAN * BKP_PLAN;
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

extern "C" size_t rr_wgrad_workspace(const rr_wgrad_desc *d) {
  if (!d) return 0;
  const Plan p = plan_of(d);
  return (size_t)p.nsplit * p.CA * p.taps * p.CB * sizeof(float);
}

extern "C" int rr_wgrad(const rr_wgrad_desc *d, const void *dy, const void *x1,
                        const void *x2, float *dw, void *ws, size_t ws_bytes,
                        rr_stream stream) {
  if (!d || !dy || !x1 || !dw) return RR_EINVAL;
  if (d->mode != RR_CONV3X3 && d->mode != RR_CONV1X1 && d->mode != RR_CONVT_UP) return RR_EINVAL;
  if (d->c_in1 % 64 || d->c_in2 % 64 || d->c_out % 64) return RR_EUNSUPPORTED;
  if (d->c_in2 > 0 && (!x2 || d->mode == RR_CONVT_UP)) return RR_EINVAL;
  const long long P = (long long)d->n * d->h * d->w;
  if (P <= 0 || P * 4 > 0x7fffffffLL) return RR_EUNSUPPORTED;
  const Plan pl = plan_of(d);
  const size_t need = (size_t)pl.nsplit * pl.CA * pl.taps * pl.CB * sizeof(float);
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
  a.fd_w = make_fastdiv((uint32_t)d->w);
  a.fd_hw = make_fastdiv((uint32_t)(d->h * d->w));
  hipStream_t st = (hipStream_t)stream;
  int rc = d->dtype == RR_BF16 ? launch_t<bf16_t>(d, pl, a, st) : launch_t<float>(d, pl, a, st);
  if (rc) return rc;
  const long long total = (long long)pl.CA * pl.CB * pl.taps;
  hipLaunchKernelGGL(wgrad_reduce, dim3(rr_grid_cap((total + 255) / 256, 8192)), dim3(256), 0, st,
                     (const float *)ws, dw, pl.CA, pl.CB, pl.taps, pl.nsplit, d->accumulate);
  RR_CHECK_LAUNCH();
  return RR_OK;
}
