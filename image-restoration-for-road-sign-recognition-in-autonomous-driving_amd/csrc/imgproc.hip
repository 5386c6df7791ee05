// imgproc.hip -- the image I/O either side of the networks (SURVEY §8f rows 2
// and 4), on device:
//
//   * rr_resize_bilinear_u8: torchvision Resize((oh, ow)) on a PIL image, i.e.
//     PIL Image.resize(BILINEAR) (17:66, 18:28-32), bit-exact: PIL's separable
//     two-pass resample with antialiasing support (filter support scaled by
//     the downscale factor), coefficients normalised in double and rounded to
//     22-bit fixed point, an 8-bit clip after each pass.  Optionally fused with
//     ToTensor (x / 255 in fp32) and Normalize ((x - mean) / std in fp32, 18:31)
//     into an NCHW fp32 batch.
//   * rr_cv_resize_linear_u8: cv2.resize(img, (ow, oh)) INTER_LINEAR, the
//     clean side of the 08 PSNR leg (08:118-119) -- OpenCV's own fixed-point
//     bilinear (resize.cpp resizeGeneric_ + HResizeLinear / VResizeLinear),
//     not Pillow's: 11-bit weights from float source coordinates, an exact
//     int32 horizontal pass, the vertical pass as the x86 SIMD body computes
//     it (VResizeLinearVec_32s8u) with the scalar 22-bit rounding on the row
//     tail; bit-equal to oracle/imgproc_cpu.cv_resize_linear (parity vs cv2
//     itself unpinned: cv2 is not installed).
//   * rr_ssim_u8: skimage structural_similarity(a, b, data_range=255,
//     channel_axis=2) (08:125): 7x7 uniform window, sample covariance
//     (49/48), K1 = .01, K2 = .03, mean of S over the interior (3-pixel border
//     cropped), mean over channels, fp64.
//
// Both are HBM-bound byte work: no MFMA, one thread per output pixel (resize)
// or per output column (SSIM), coalesced along the innermost NHWC axis.
#include "common.h"

#include <cmath>

namespace {

// ---------------------------------------------------------------- resize ----
constexpr int RS_PREC = 22;        // PIL PRECISION_BITS = 32 - 8 - 2
constexpr int RS_MAXK = 255;       // taps per output (downscale up to 127x)

struct RsAxis {
  int in_size, out_size, ksize;
  int *bounds;                     // [out][2]: first tap, tap count
  int *kk;                         // [out][ksize] fixed-point coefficients
};

// PIL precompute_coeffs + normalize_coeffs_8bpc (Resample.c), evaluated in
// the same double operations in the same order; contraction into FMA would
// change the rounding, so it is off for this function.
__device__ void rs_coeffs_one(const RsAxis &ax, int xx) {
#pragma clang fp contract(off)
  const double scale = (double)ax.in_size / ax.out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;                  // bilinear support 1.0
  const double center = 0.0 + (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > ax.in_size) xmax = ax.in_size;
  xmax -= xmin;
  // the filter value of tap x (evaluated twice: sum first, then normalise --
  // the same doubles both times, and no private array in scratch)
  auto tap = [&](int x) {
    double t = ((double)(x + xmin) - center + 0.5) * ss;
    t = t < 0.0 ? -t : t;
    return t < 1.0 ? 1.0 - t : 0.0;
  };
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) ww += tap(x);
  int *o = ax.kk + (long long)xx * ax.ksize;
  for (int x = 0; x < ax.ksize; ++x) {
    double v = 0.0;
    if (x < xmax) v = ww != 0.0 ? tap(x) / ww : tap(x);
    o[x] = v < 0 ? (int)(-0.5 + v * (double)(1 << RS_PREC)) : (int)(0.5 + v * (double)(1 << RS_PREC));
  }
  ax.bounds[2 * xx] = xmin;
  ax.bounds[2 * xx + 1] = xmax;
}

__global__ void rs_coeffs_kernel(RsAxis h, RsAxis v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < h.out_size) rs_coeffs_one(h, i);
  else if (i < h.out_size + v.out_size) rs_coeffs_one(v, i - h.out_size);
}

__device__ __forceinline__ int rs_clip8(int s) {          // PIL clip8: lookups[s >> 22]
  const int v = s >> RS_PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// horizontal pass over source rows [y_first, y_first + rows): [n][h][w][C] ->
// tmp [n][rows][ow][C]
template <int C>
__global__ void rs_horiz_kernel(int n, int h, int w, int ow, int y_first, int rows, int ksize,
                                const int *__restrict__ bounds, const int *__restrict__ kk,
                                const uint8_t *__restrict__ in, uint8_t *__restrict__ tmp) {
  const long long total = (long long)n * rows * ow;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ox = (int)(i % ow);
    const long long r = i / ow;                    // n * rows + row
    const int img = (int)(r / rows), y = (int)(r % rows) + y_first;
    const int xmin = bounds[2 * ox], xcnt = bounds[2 * ox + 1];
    const int *k = kk + (long long)ox * ksize;
    const uint8_t *src = in + (((long long)img * h + y) * w + xmin) * C;
    int s[C];
#pragma unroll
    for (int c = 0; c < C; ++c) s[c] = 1 << (RS_PREC - 1);
    for (int x = 0; x < xcnt; ++x) {
      const int kx = k[x];
#pragma unroll
      for (int c = 0; c < C; ++c) s[c] += (int)src[x * C + c] * kx;
    }
    uint8_t *dst = tmp + i * C;
#pragma unroll
    for (int c = 0; c < C; ++c) dst[c] = (uint8_t)rs_clip8(s[c]);
  }
}

struct RsNorm { float mean[4], std[4]; };

// vertical pass: tmp [n][rows][ow][C] -> u8 [n][oh][ow][C] (MODE 0) or fp32
// NCHW ToTensor (+ Normalize) (MODE 1)
template <int C, int MODE>
__global__ void rs_vert_kernel(int n, int rows, int oh, int ow, int ksize, int y_first,
                               const int *__restrict__ bounds, const int *__restrict__ kk,
                               const uint8_t *__restrict__ tmp, void *__restrict__ out, RsNorm nm,
                               int normalize) {
  const long long total = (long long)n * oh * ow;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ox = (int)(i % ow);
    const long long r = i / ow;
    const int img = (int)(r / oh), oy = (int)(r % oh);
    const int ymin = bounds[2 * oy] - y_first, ycnt = bounds[2 * oy + 1];
    const int *k = kk + (long long)oy * ksize;
    const uint8_t *src = tmp + (((long long)img * rows + ymin) * ow + ox) * C;
    int s[C];
#pragma unroll
    for (int c = 0; c < C; ++c) s[c] = 1 << (RS_PREC - 1);
    for (int y = 0; y < ycnt; ++y) {
      const int ky = k[y];
#pragma unroll
      for (int c = 0; c < C; ++c) s[c] += (int)src[(long long)y * ow * C + c] * ky;
    }
    if constexpr (MODE == 0) {
      uint8_t *dst = (uint8_t *)out + i * C;
#pragma unroll
      for (int c = 0; c < C; ++c) dst[c] = (uint8_t)rs_clip8(s[c]);
    } else {
      float *dst = (float *)out;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float v = (float)rs_clip8(s[c]) / 255.0f;                 // ToTensor: .div(255)
        if (normalize) v = (v - nm.mean[c]) / nm.std[c];          // Normalize: sub_, div_
        dst[(((long long)img * C + c) * oh + oy) * ow + ox] = v;
      }
    }
  }
}

// same-size "resize": Pillow returns a copy of the image (Image.resize with
// size == self.size), so the passes reduce to the copy / ToTensor (+
// Normalize) of the input -- one pass instead of horiz + vert + coefficients
template <int C, int MODE>
__global__ void rs_same_kernel(long long npix, int hw, const uint8_t *__restrict__ in,
                               void *__restrict__ out, RsNorm nm, int normalize) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < npix;
       i += (long long)gridDim.x * blockDim.x) {
    const uint8_t *src = in + i * C;
    if constexpr (MODE == 0) {
      uint8_t *dst = (uint8_t *)out + i * C;
#pragma unroll
      for (int c = 0; c < C; ++c) dst[c] = src[c];
    } else {
      const long long img = i / hw, px = i - img * hw;
      float *dst = (float *)out;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float v = (float)src[c] / 255.0f;                           // ToTensor: .div(255)
        if (normalize) v = (v - nm.mean[c]) / nm.std[c];          // Normalize: sub_, div_
        dst[(img * C + c) * hw + px] = v;
      }
    }
  }
}

struct RsPlan {
  int kh, kv, y_first, rows;
  size_t off_bh, off_kh, off_bv, off_kv, off_tmp, total;
};

// host mirror of the bound computation for the rows the vertical pass reads
// (PIL ybox_first / ybox_last); same double expressions as rs_coeffs_one
static void rs_vbox(int in_size, int out_size, int *first, int *last) {
  const double scale = (double)in_size / out_size;
  const double support = scale < 1.0 ? 1.0 : scale;
  auto lo = [&](int yy) {
    const double c = 0.0 + (yy + 0.5) * scale;
    int a = (int)(c - support + 0.5);
    return a < 0 ? 0 : a;
  };
  auto hi = [&](int yy) {
    const double c = 0.0 + (yy + 0.5) * scale;
    int b = (int)(c + support + 0.5);
    return b > in_size ? in_size : b;
  };
  *first = lo(0);
  *last = hi(out_size - 1);   // bounds[last] start + count = clamped xmax
}

static int rs_ksize(int in_size, int out_size) {
  const double scale = (double)in_size / out_size;
  const double support = scale < 1.0 ? 1.0 : scale;
  return (int)std::ceil(support) * 2 + 1;
}

static bool rs_plan(int n, int h, int w, int c, int oh, int ow, RsPlan *p) {
  if (n <= 0 || h <= 0 || w <= 0 || oh <= 0 || ow <= 0 || c < 1 || c > 4) return false;
  p->kh = rs_ksize(w, ow);
  p->kv = rs_ksize(h, oh);
  if (p->kh > RS_MAXK || p->kv > RS_MAXK) return false;
  int f, l;
  rs_vbox(h, oh, &f, &l);
  p->y_first = f;
  p->rows = l - f;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t o = 0;
  p->off_bh = o; o = al(o + (size_t)ow * 2 * 4);
  p->off_kh = o; o = al(o + (size_t)ow * p->kh * 4);
  p->off_bv = o; o = al(o + (size_t)oh * 2 * 4);
  p->off_kv = o; o = al(o + (size_t)oh * p->kv * 4);
  p->off_tmp = o; o = al(o + (size_t)n * p->rows * ow * c);
  p->total = o;
  return true;
}

// ------------------------------------------------------------------ SSIM ----
constexpr int SS_T = 256;

// one workgroup per (image, channel): thread = output column, sliding 7-row
// window of exact integer 7x7 sums (x, y, x^2, y^2, xy); S in fp64; fixed-order
// reduction -> per-(image, channel) mean of S over the cropped interior
__global__ __launch_bounds__(SS_T) void ssim_kernel(int h, int w, int C, const uint8_t *__restrict__ a,
                                                    const uint8_t *__restrict__ b,
                                                    double *__restrict__ chan_mean) {
  const int img = blockIdx.x / C, ch = blockIdx.x % C;
  const uint8_t *pa = a + (long long)img * h * w * C + ch;
  const uint8_t *pb = b + (long long)img * h * w * C + ch;
  const double C1 = (0.01 * 255.0) * (0.01 * 255.0), C2 = (0.03 * 255.0) * (0.03 * 255.0);
  const double cov_norm = 49.0 / 48.0;
  double acc = 0.0;
  for (int cx = 3 + threadIdx.x; cx < w - 3; cx += SS_T) {
    auto hsum = [&](int y, int &sx, int &sy, int &sxx, int &syy, int &sxy) {
      sx = sy = sxx = syy = sxy = 0;
      const long long base = ((long long)y * w + cx - 3) * C;
#pragma unroll
      for (int d = 0; d < 7; ++d) {
        const int x = pa[base + d * C], y2 = pb[base + d * C];
        sx += x; sy += y2; sxx += x * x; syy += y2 * y2; sxy += x * y2;
      }
    };
    int vx = 0, vy = 0, vxx = 0, vyy = 0, vxy = 0;
    for (int y = 0; y < h; ++y) {
      int sx, sy, sxx, syy, sxy;
      hsum(y, sx, sy, sxx, syy, sxy);
      vx += sx; vy += sy; vxx += sxx; vyy += syy; vxy += sxy;
      if (y >= 7) {
        hsum(y - 7, sx, sy, sxx, syy, sxy);
        vx -= sx; vy -= sy; vxx -= sxx; vyy -= syy; vxy -= sxy;
      }
      if (y >= 6) {
        const double ux = vx / 49.0, uy = vy / 49.0;
        const double uxx = vxx / 49.0, uyy = vyy / 49.0, uxy = vxy / 49.0;
        const double sxv = cov_norm * (uxx - ux * ux);
        const double syv = cov_norm * (uyy - uy * uy);
        const double sxyv = cov_norm * (uxy - ux * uy);
        const double A1 = 2 * ux * uy + C1, A2 = 2 * sxyv + C2;
        const double B1 = ux * ux + uy * uy + C1, B2 = sxv + syv + C2;
        acc += (A1 * A2) / (B1 * B2);
      }
    }
  }
  __shared__ double red[SS_T];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = SS_T / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) chan_mean[blockIdx.x] = red[0] / ((double)(h - 6) * (w - 6));
}

// ---------------------------------------------------------- cv resize ----
// resize.cpp's coefficient of output coordinate d: float source position
// (d + 0.5) * scale - 0.5 evaluated in double then rounded to float (no FMA:
// contraction would change the rounding), its floor and fraction
__device__ __forceinline__ void cvr_coord(int d, double scale, int *i, float *f) {
#pragma clang fp contract(off)
  const double v = ((double)d + 0.5) * scale - 0.5;
  const float fv = (float)v;
  const float fl = floorf(fv);
  *i = (int)fl;
  *f = fv - fl;
}

__device__ __forceinline__ int cvr_round(float v) { return __float2int_rn(v); }   // cvRound

// one thread per output pixel, C channels; vec_end = first row element
// (x * C + ch) of the scalar tail
template <int C>
__global__ void cv_resize_linear_kernel(int n, int h, int w, int oh, int ow, double sx_scale,
                                        double sy_scale, int vec_end,
                                        const uint8_t *__restrict__ in, uint8_t *__restrict__ out) {
#pragma clang fp contract(off)
  const long long total = (long long)n * oh * ow;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < total;
       q += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(q % ow);
    const long long r = q / ow;
    const int y = (int)(r % oh);
    const int im = (int)(r / oh);
    int sx, sy;
    float fx, fy;
    cvr_coord(x, sx_scale, &sx, &fx);
    if (sx < 0) { sx = 0; fx = 0.f; }
    if (sx >= w - 1) { sx = w - 1; fx = 0.f; }
    const int a0 = cvr_round((1.f - fx) * 2048.f), a1 = cvr_round(fx * 2048.f);
    const int sx1 = sx + 1 < w ? sx + 1 : w - 1;
    cvr_coord(y, sy_scale, &sy, &fy);
    const int b0 = cvr_round((1.f - fy) * 2048.f), b1 = cvr_round(fy * 2048.f);
    const int r0 = sy < 0 ? 0 : (sy > h - 1 ? h - 1 : sy);
    const int r1 = sy + 1 < 0 ? 0 : (sy + 1 > h - 1 ? h - 1 : sy + 1);
    const uint8_t *p0 = in + ((long long)im * h + r0) * w * C;
    const uint8_t *p1 = in + ((long long)im * h + r1) * w * C;
    uint8_t *o = out + q * C;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int s0 = (int)p0[sx * C + c] * a0 + (int)p0[sx1 * C + c] * a1;
      const int s1 = (int)p1[sx * C + c] * a0 + (int)p1[sx1 * C + c] * a1;
      int v;
      if (x * C + c < vec_end) {
        // v_mul_hi on the int16-packed S >> 4, then v_rshr_pack_u<2>
        v = ((((s0 >> 4) * b0) >> 16) + (((s1 >> 4) * b1) >> 16) + 2) >> 2;
      } else {
        v = (int)(((long long)s0 * b0 + (long long)s1 * b1 + (1LL << 21)) >> 22);
      }
      o[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
  }
}

__global__ void ssim_chan_mean_kernel(int n, int C, const double *__restrict__ chan_mean,
                                      double *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int c = 0; c < C; ++c) s += chan_mean[(long long)i * C + c];
  out[i] = s / C;
}

}  // namespace

int rr_copy_bytes(void *dst, const void *src, size_t bytes, hipStream_t st);   // misc.hip

extern "C" size_t rr_resize_workspace(int n, int h, int w, int c, int oh, int ow) {
  RsPlan p;
  return rs_plan(n, h, w, c, oh, ow, &p) ? p.total : 0;
}

extern "C" int rr_resize_bilinear_u8(int n, int h, int w, int c, int oh, int ow, const uint8_t *in,
                                     int out_kind, const float *mean, const float *std, void *out,
                                     void *ws, size_t ws_bytes, rr_stream stream) {
  RsPlan p;
  if (!in || !out || !ws || (out_kind != 0 && out_kind != 1)) return RR_EINVAL;
  if (!rs_plan(n, h, w, c, oh, ow, &p)) return RR_EUNSUPPORTED;
  if (ws_bytes < p.total) return RR_EWORKSPACE;
  if ((mean == nullptr) != (std == nullptr) || (mean && out_kind != 1)) return RR_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (oh == h && ow == w) {
    RsNorm nm{};
    for (int i = 0; i < c; ++i) {
      nm.mean[i] = mean ? mean[i] : 0.f;
      nm.std[i] = std ? std[i] : 1.f;
    }
    const long long np = (long long)n * h * w;
    const dim3 g(rr_grid_cap((np + 255) / 256, 8192)), b(256);
#define RS_SAME(CC)                                                                                 \
  if (out_kind == 0) hipLaunchKernelGGL((rs_same_kernel<CC, 0>), g, b, 0, st, np, h * w, in, out, nm, 0); \
  else hipLaunchKernelGGL((rs_same_kernel<CC, 1>), g, b, 0, st, np, h * w, in, out, nm, mean != nullptr);
    switch (c) {
      case 1: RS_SAME(1) break;
      case 2: RS_SAME(2) break;
      case 3: RS_SAME(3) break;
      default: RS_SAME(4) break;
    }
#undef RS_SAME
    RR_CHECK_LAUNCH();
    return RR_OK;
  }
  char *base = (char *)ws;
  RsAxis ah{w, ow, p.kh, (int *)(base + p.off_bh), (int *)(base + p.off_kh)};
  RsAxis av{h, oh, p.kv, (int *)(base + p.off_bv), (int *)(base + p.off_kv)};
  hipLaunchKernelGGL(rs_coeffs_kernel, dim3((ow + oh + 63) / 64), dim3(64), 0, st, ah, av);
  RR_CHECK_LAUNCH();
  uint8_t *tmp = (uint8_t *)(base + p.off_tmp);
  const long long th = (long long)n * p.rows * ow, tv = (long long)n * oh * ow;
  const dim3 gh(rr_grid_cap((th + 255) / 256, 8192)), gv(rr_grid_cap((tv + 255) / 256, 8192)), b(256);
  RsNorm nm{};
  for (int i = 0; i < c; ++i) {
    nm.mean[i] = mean ? mean[i] : 0.f;
    nm.std[i] = std ? std[i] : 1.f;
  }
  const int norm = mean != nullptr;
#define RS_LAUNCH(CC)                                                                              \
  hipLaunchKernelGGL(rs_horiz_kernel<CC>, gh, b, 0, st, n, h, w, ow, p.y_first, p.rows, p.kh,    \
                     ah.bounds, ah.kk, in, tmp);                                                   \
  if (out_kind == 0)                                                                               \
    hipLaunchKernelGGL((rs_vert_kernel<CC, 0>), gv, b, 0, st, n, p.rows, oh, ow, p.kv, p.y_first, \
                       av.bounds, av.kk, tmp, out, nm, norm);                                      \
  else                                                                                             \
    hipLaunchKernelGGL((rs_vert_kernel<CC, 1>), gv, b, 0, st, n, p.rows, oh, ow, p.kv, p.y_first, \
                       av.bounds, av.kk, tmp, out, nm, norm);
  switch (c) {
    case 1: RS_LAUNCH(1) break;
    case 2: RS_LAUNCH(2) break;
    case 3: RS_LAUNCH(3) break;
    default: RS_LAUNCH(4) break;
  }
#undef RS_LAUNCH
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" int rr_cv_resize_linear_u8(int n, int h, int w, int c, int oh, int ow,
                                      const uint8_t *in, uint8_t *out, int simd_lanes,
                                      rr_stream stream) {
  if (n < 0 || h <= 0 || w <= 0 || oh <= 0 || ow <= 0 || c < 1 || c > 4) return RR_EINVAL;
  if (simd_lanes <= 0) simd_lanes = 16;
  if ((simd_lanes & 1) != 0) return RR_EINVAL;
  if (n == 0) return RR_OK;
  if (!in || !out) return RR_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (oh == h && ow == w) {                               // cv::resize: same size -> copy
    return rr_copy_bytes(out, in, (size_t)n * h * w * c, st);   // (a kernel: graph-safe, misc.hip)
  }
  // hal::resize: scale = 1 / inv_scale, inv_scale = dst / src (double)
  const double sxs = 1.0 / ((double)ow / (double)w), sys = 1.0 / ((double)oh / (double)h);
  // VResizeLinearVec_32s8u: x <= width - lanes in full vectors, then
  // x < width - lanes / 2 in half vectors; the rest scalar
  const int width = ow * c;
  int ve = (width / simd_lanes) * simd_lanes;
  while (ve < width - simd_lanes / 2) ve += simd_lanes / 2;
  const long long total = (long long)n * oh * ow;
  const dim3 g(rr_grid_cap((total + 255) / 256, 8192)), b(256);
  switch (c) {
    case 1: hipLaunchKernelGGL(cv_resize_linear_kernel<1>, g, b, 0, st, n, h, w, oh, ow, sxs, sys, ve, in, out); break;
    case 2: hipLaunchKernelGGL(cv_resize_linear_kernel<2>, g, b, 0, st, n, h, w, oh, ow, sxs, sys, ve, in, out); break;
    case 3: hipLaunchKernelGGL(cv_resize_linear_kernel<3>, g, b, 0, st, n, h, w, oh, ow, sxs, sys, ve, in, out); break;
    default: hipLaunchKernelGGL(cv_resize_linear_kernel<4>, g, b, 0, st, n, h, w, oh, ow, sxs, sys, ve, in, out); break;
  }
  RR_CHECK_LAUNCH();
  return RR_OK;
}

extern "C" size_t rr_ssim_workspace(int n, int c) {
  return n > 0 && c > 0 ? (size_t)n * c * sizeof(double) : 0;
}

extern "C" int rr_ssim_u8(int n, int h, int w, int c, const uint8_t *a, const uint8_t *b, double *out,
                          void *ws, size_t ws_bytes, rr_stream stream) {
  if (!a || !b || !out || !ws || n <= 0 || c <= 0) return RR_EINVAL;
  if (h < 7 || w < 7) return RR_EINVAL;                     // skimage: win_size > image side
  if (ws_bytes < rr_ssim_workspace(n, c)) return RR_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  double *cm = (double *)ws;
  hipLaunchKernelGGL(ssim_kernel, dim3(n * c), dim3(SS_T), 0, st, h, w, c, a, b, cm);
  RR_CHECK_LAUNCH();
  hipLaunchKernelGGL(ssim_chan_mean_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, c, cm, out);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

// ------------------------------------------------------------ distortion ----
// The dynamic distortion generator 14:31-64 (fog -> noise -> motion blur, each
// drawn per image) and the fixed compound variant 16:14-37 (blur -> fog ->
// noise), per image on device, with the reference's numpy dtype semantics:
//   img / 255 in fp32; fog out * f32(t) + f32(A (1 - t)) in fp32; noise added
//   in fp64 (np.random.normal is float64, so the image becomes float64);
//   clip(x * 255, 0, 255).astype(uint8) truncates; cv2.filter2D on uint8 with
//   the fp32-converted kernel: fp32 sum over the taps in row-major order,
//   BORDER_REFLECT_101, anchor (k / 2, k / 2), round half to even, saturate.
// Noise: the caller's fp64 field (parity runs) or Philox4x32-10 normals
// (Box-Muller in fp64) keyed by (seed, element index).

struct DistCfg {
  int n, h, w, c, mode;                 // mode 0: 14:31-64 order, 1: 16:14-37 order
  const uint8_t *in;
  uint8_t *out, *tmp;
  const rr_distort_param *prm;
  const float *taps;                    // [n][RR_DISTORT_KMAX^2], row-major
  const double *noise;                  // [n][h][w][c] or null -> Philox
  unsigned long long seed;
  const int *tap_idx;                   // null, or [n]: image i's taps are taps + tap_idx[i] * KMAX^2
  const unsigned long long *seed_dev;   // null, or the Philox seed in device memory
};

__device__ __forceinline__ unsigned long long dist_seed(const DistCfg &a) {
  return a.seed_dev ? *a.seed_dev : a.seed;
}

__device__ __forceinline__ void philox_round(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3,
                                             uint32_t k0, uint32_t k1) {
  const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
  const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
  const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
  const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
  const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
  c0 = n0; c1 = l1; c2 = n2; c3 = l0;
}

// standard normal for element e (Philox4x32-10, two 24-bit uniforms,
// Box-Muller in fp32: np.random.normal's stream cannot be reproduced anyway,
// and the fp32 transcendentals cost a fraction of the fp64 library ones --
// the noise feeds an fp64 add and a uint8 truncation; |z| <= 5.8)
__device__ double philox_normal(unsigned long long seed, unsigned long long e) {
  uint32_t c0 = (uint32_t)e, c1 = (uint32_t)(e >> 32), c2 = 0x9E3779B9u, c3 = 0;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  const float u1 = (float)((c0 >> 8) + 1) * 0x1p-24f;          // (0, 1]
  const float u2 = (float)(c2 >> 8) * 0x1p-24f;                // [0, 1)
  return (double)(sqrtf(-2.f * logf(u1)) * cosf(6.28318530717958648f * u2));
}

__device__ __forceinline__ uint8_t trunc_u8(double v) {    // np.clip(v, 0, 255).astype(uint8)
  v = v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v);
  return (uint8_t)(int)v;
}
__device__ __forceinline__ uint8_t trunc_u8f(float v) {
  v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
  return (uint8_t)(int)v;
}

// fog then noise on x = img / 255 (fp32); returns clip(x * 255).astype(u8)
// in the dtype the reference holds at that point
__device__ __forceinline__ uint8_t fog_noise(const DistCfg &a, const rr_distort_param &p, float x,
                                             long long e) {
#pragma clang fp contract(off)
  if (p.flags & RR_DISTORT_FOG) x = x * p.fog_mul + p.fog_add;
  if (p.flags & RR_DISTORT_NOISE) {
    const double nz = a.noise ? a.noise[e] : p.sigma * philox_normal(dist_seed(a), (unsigned long long)e);
    return trunc_u8(((double)x + nz) * 255.0);
  }
  return trunc_u8f(x * 255.f);
}

__device__ __forceinline__ int reflect101(int p, int len) {
  if (len == 1) return 0;
  while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - 2 - p;
  return p;
}

// stage 1 (per element): mode 0: fog/noise -> u8 (the blur input, or the
// output if no blur); mode 1: (img / 255 * 255).astype(u8), the blur input
__global__ void distort_pre_kernel(DistCfg a) {
#pragma clang fp contract(off)
  const long long per = (long long)a.h * a.w * a.c, total = per * a.n;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int img = (int)(e / per);
    const rr_distort_param p = a.prm[img];
    const float x = (float)a.in[e] / 255.0f;
    const bool blur = p.flags & RR_DISTORT_BLUR;
    uint8_t v;
    if (a.mode == 0) v = fog_noise(a, p, x, e);
    else v = trunc_u8f(x * 255.f);
    if (blur) a.tmp[e] = v;
    else if (a.mode == 0) a.out[e] = v;
    else a.out[e] = fog_noise(a, p, (float)v / 255.0f, e);
  }
}

// stage 2 (blurred images only): filter2D of tmp, then mode 0: the u8 result
// ((t / 255) * 255 truncated), mode 1: fog + noise on it
__device__ __forceinline__ void blur_store(const DistCfg &a, const rr_distort_param &p, long long q,
                                           const float *s) {
#pragma clang fp contract(off)
  for (int c = 0; c < a.c; ++c) {
    float r = rintf(s[c]);                                   // saturate_cast<uchar>: cvRound
    r = r < 0.f ? 0.f : (r > 255.f ? 255.f : r);
    const long long e = q * a.c + c;
    const float t = (float)(int)r / 255.0f;
    a.out[e] = a.mode == 0 ? trunc_u8f(t * 255.f) : fog_noise(a, p, t, e);
  }
}

__global__ void distort_blur_kernel(DistCfg a) {
#pragma clang fp contract(off)
  const long long hw = (long long)a.h * a.w, total = hw * a.n;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < total;
       q += (long long)gridDim.x * blockDim.x) {
    const int img = (int)(q / hw);
    const rr_distort_param p = a.prm[img];
    if (!(p.flags & RR_DISTORT_BLUR)) continue;
    const int rem = (int)(q - (long long)img * hw), y = rem / a.w, x = rem % a.w;
    const int k = p.ksize, anc = k / 2;
    const float *kt = a.taps + (long long)(a.tap_idx ? a.tap_idx[img] : img) * RR_DISTORT_KMAX * RR_DISTORT_KMAX;
    const uint8_t *src = a.tmp + (long long)img * hw * a.c;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < k; ++i) {
      const int yy = reflect101(y + i - anc, a.h);
      for (int j = 0; j < k; ++j) {
        const float kv = kt[i * RR_DISTORT_KMAX + j];
        if (kv == 0.f) continue;                             // cv2 drops zero taps
        const int xx = reflect101(x + j - anc, a.w);
        const uint8_t *px = src + ((long long)yy * a.w + xx) * a.c;
        for (int c = 0; c < a.c; ++c) s[c] = s[c] + kv * (float)px[c];
      }
    }
    blur_store(a, p, q, s);
  }
}

// the same with the image's nonzero taps compacted into LDS first (row-major,
// so the sums run in the same order: bit-identical) -- for h * w a multiple
// of 256, where a workgroup's 256 pixels always belong to one image: the
// per-pixel loop then visits the ~k..2k nonzero taps of the rotated line
// kernel instead of testing all k * k, with no per-tap global loads
//
// The source rows the 256 pixels read (their row span + k - 1, reflect-101
// applied at staging, columns -anc .. w - 1 + k - 1 - anc) are staged in LDS
// when they fit: the tap loop then reads bytes at (row, x + j) with no
// reflection and no global load (same values, same order: bit-identical)
#define RR_BLUR_LDS 24576
__global__ __launch_bounds__(256) void distort_blur_tiled_kernel(DistCfg a) {
#pragma clang fp contract(off)
  __shared__ float tv[RR_DISTORT_KMAX * RR_DISTORT_KMAX];
  __shared__ int ti[RR_DISTORT_KMAX * RR_DISTORT_KMAX];
  __shared__ int wcount[4];
  __shared__ uint8_t simg[RR_BLUR_LDS];
  const long long hw = (long long)a.h * a.w, total = hw * a.n;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (long long q0 = blockIdx.x * 256LL; q0 < total; q0 += (long long)gridDim.x * 256) {
    const int img = (int)(q0 / hw);                          // uniform: 256 | hw
    const rr_distort_param p = a.prm[img];
    if (!(p.flags & RR_DISTORT_BLUR)) continue;              // uniform
    const int k = p.ksize, anc = k / 2;
    const float *kt = a.taps + (long long)(a.tap_idx ? a.tap_idx[img] : img) * RR_DISTORT_KMAX * RR_DISTORT_KMAX;
    const int i = t / (k > 0 ? k : 1), j = t - i * (k > 0 ? k : 1);
    const float kv = t < k * k ? kt[i * RR_DISTORT_KMAX + j] : 0.f;
    const bool nz = kv != 0.f;                               // cv2 drops zero taps
    const unsigned long long m = __ballot(nz);
    const int pos = __popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();                                         // the previous image's list is read
    if (lane == 0) wcount[wv] = __popcll(m);
    const uint8_t *src = a.tmp + (long long)img * hw * a.c;
    const int rem0 = (int)(q0 - (long long)img * hw);
    const int ya = rem0 / a.w, yb = (rem0 + 255) / a.w;      // row span of the 256 pixels
    const int pw = a.w + k - 1, nr = yb - ya + k;             // staged columns / rows
    const bool lds = nr * pw * a.c <= RR_BLUR_LDS;           // uniform
    if (lds) {
      const int rowb = pw * a.c;
      for (int e = t; e < nr * rowb; e += 256) {
        const int r = e / rowb, rest = e - r * rowb;
        const int cx = rest / a.c, ch = rest - cx * a.c;
        const int yy = reflect101(ya - anc + r, a.h), xx = reflect101(cx - anc, a.w);
        simg[e] = src[((long long)yy * a.w + xx) * a.c + ch];
      }
    }
    __syncthreads();
    int off = 0;
    for (int u = 0; u < wv; ++u) off += wcount[u];
    if (nz) { tv[off + pos] = kv; ti[off + pos] = (i << 8) | j; }
    const int nt = wcount[0] + wcount[1] + wcount[2] + wcount[3];
    __syncthreads();
    const long long q = q0 + t;
    const int rem = (int)(q - (long long)img * hw), y = rem / a.w, x = rem % a.w;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    if (lds) {
      const uint8_t *base = simg + ((y - ya) * pw + x) * a.c;
      for (int u = 0; u < nt; ++u) {
        const int ij = ti[u];
        const float w = tv[u];
        const uint8_t *px = base + ((ij >> 8) * pw + (ij & 255)) * a.c;
        for (int c = 0; c < a.c; ++c) s[c] = s[c] + w * (float)px[c];
      }
    } else {
      for (int u = 0; u < nt; ++u) {
        const int ij = ti[u];
        const float w = tv[u];
        const int yy = reflect101(y + (ij >> 8) - anc, a.h), xx = reflect101(x + (ij & 255) - anc, a.w);
        const uint8_t *px = src + ((long long)yy * a.w + xx) * a.c;
        for (int c = 0; c < a.c; ++c) s[c] = s[c] + w * (float)px[c];
      }
    }
    blur_store(a, p, q, s);
  }
}

static void launch_blur(const DistCfg &a, long long tp, hipStream_t st) {
  // the LDS-tiled form where whole 256-pixel tiles fit (RR_PATH
  // blur_tiled=0: the per-pixel kernel, tests)
  if (((long long)a.h * a.w) % 256 == 0 && a.c <= 4 && rr_path("blur_tiled", 1))
    hipLaunchKernelGGL(distort_blur_tiled_kernel, dim3(rr_grid_cap((tp + 255) / 256, 8192)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(distort_blur_kernel, dim3(rr_grid_cap((tp + 255) / 256, 8192)), dim3(256), 0, st, a);
}

// ---------------------------------------------------- on-device draws ----
// The per-image draws of apply_random_distortions (14:36-58) made on device,
// so the whole data step is graph-capturable: the same distributions as the
// reference's Python `random` calls (fog with p 0.5, intensity U(0.3, 0.7),
// t = 1 - intensity * U(0.8, 1.2), A = 0.9; noise with p 0.5, var U(0.01,
// 0.03); blur with p 0.5, degree randint(5, 15), angle randint(0, 360)), drawn
// from Philox4x32-10 keyed by (seed, step) with the image index as counter
// (the reference's stream is unseeded, so only the distributions can match).
// The step counter lives in device memory and advances once per call; the
// blur kernel of (degree, angle) is an index into a table of all 11 x 361
// kernels built once on the host by rr_motion_blur_kernel.
constexpr int DRAW_DEG0 = 5, DRAW_NDEG = 11, DRAW_NANG = 361;

__device__ __forceinline__ void philox4(uint32_t c[4], unsigned long long key) {
  uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c[0], c[1], c[2], c[3], k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ double u01(uint32_t hi, uint32_t lo) {       // [0, 1), 53 bits
  return ((((unsigned long long)hi << 21) ^ lo) & ((1ull << 53) - 1)) * 0x1p-53;
}

__global__ __launch_bounds__(256) void distort_draw_kernel(int n, unsigned long long seed,
                                                           long long *step, rr_distort_param *prm,
                                                           int *tap_idx, unsigned long long *noise_seed) {
#pragma clang fp contract(off)
  const long long s = *step;
  const unsigned long long key = seed ^ (0x9E3779B97F4A7C15ull * (unsigned long long)(s + 1));
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t a[4] = {(uint32_t)i, 0u, 0x5EED0001u, 0u}, b[4] = {(uint32_t)i, 1u, 0x5EED0001u, 0u};
    philox4(a, key);
    philox4(b, key);
    const double r_fog = u01(a[0], a[1]), r_int = u01(a[2], a[3]);
    const double r_t = u01(b[0], b[1]), r_noise = u01(b[2], b[3]);
    uint32_t c[4] = {(uint32_t)i, 2u, 0x5EED0001u, 0u}, d[4] = {(uint32_t)i, 3u, 0x5EED0001u, 0u};
    philox4(c, key);
    philox4(d, key);
    const double r_var = u01(c[0], c[1]), r_blur = u01(c[2], c[3]);
    const double r_deg = u01(d[0], d[1]), r_ang = u01(d[2], d[3]);
    rr_distort_param p;
    p.sigma = 0.0;
    p.fog_mul = 1.0f;
    p.fog_add = 0.0f;
    p.flags = 0;
    p.ksize = 0;
    int ti = 0;
    if (r_fog < 0.5) {
      const double intensity = 0.3 + (0.7 - 0.3) * r_int;
      const double t = 1.0 - intensity * (0.8 + (1.2 - 0.8) * r_t);
      p.flags |= RR_DISTORT_FOG;
      p.fog_mul = (float)t;
      p.fog_add = (float)(0.9 * (1.0 - t));
    }
    if (r_noise < 0.5) {
      const double var = 0.01 + (0.03 - 0.01) * r_var;
      p.flags |= RR_DISTORT_NOISE;
      p.sigma = sqrt(var);
    }
    if (r_blur < 0.5) {
      const int deg = DRAW_DEG0 + (int)(r_deg * DRAW_NDEG);
      const int ang = (int)(r_ang * DRAW_NANG);
      p.flags |= RR_DISTORT_BLUR;
      p.ksize = deg;
      ti = (deg - DRAW_DEG0) * DRAW_NANG + ang;
    }
    prm[i] = p;
    tap_idx[i] = ti;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t e[4] = {0xFFFFFFFFu, 0u, 0x5EED0002u, 0u};
    philox4(e, key);
    *noise_seed = ((unsigned long long)e[0] << 32) | e[1];
    *step = s + 1;
  }
}

extern "C" size_t rr_distort_workspace(int n, int h, int w, int c) {
  return n > 0 && h > 0 && w > 0 && c > 0 ? (size_t)n * h * w * c : 0;
}

extern "C" int rr_distort_u8(int n, int h, int w, int c, int mode, const uint8_t *in, uint8_t *out,
                             const rr_distort_param *params, const float *taps, const double *noise,
                             unsigned long long seed, void *ws, size_t ws_bytes, rr_stream stream) {
  if (!in || !out || !params || !taps || !ws || n <= 0 || h <= 0 || w <= 0) return RR_EINVAL;
  if (c < 1 || c > 4 || (mode != 0 && mode != 1)) return RR_EINVAL;
  if (ws_bytes < rr_distort_workspace(n, h, w, c)) return RR_EWORKSPACE;
  DistCfg a{n, h, w, c, mode, in, out, (uint8_t *)ws, params, taps, noise, seed, nullptr, nullptr};
  hipStream_t st = (hipStream_t)stream;
  const long long te = (long long)n * h * w * c, tp = (long long)n * h * w;
  hipLaunchKernelGGL(distort_pre_kernel, dim3(rr_grid_cap((te + 255) / 256, 8192)), dim3(256), 0, st, a);
  RR_CHECK_LAUNCH();
  launch_blur(a, tp, st);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

// cv2.getRotationMatrix2D((k / 2, k / 2), angle, 1) + cv2.warpAffine of
// np.diag(np.ones(k)) (INTER_LINEAR, BORDER_CONSTANT 0, dsize (k, k)) / k,
// converted to fp32 as filter2D does (14:55-59, 16:20-21).  Host code: the
// reference builds this kernel on the host per image too; it is <= 225 taps.
// warpAffine: inverted matrix, 10-bit fixed-point source coordinates rounded
// half-even, 1/32-pixel interpolation table of fp32 bilinear weights.
extern "C" int rr_motion_blur_kernel(int k, int angle, float *taps) {
  if (!taps || k < 1 || k > RR_DISTORT_KMAX) return RR_EINVAL;
  const double cx = (float)(k / 2.0), cy = cx;
  const double ang = angle * 3.14159265358979323846 / 180.0;
  const double alpha = std::cos(ang) * 1.0, beta = std::sin(ang) * 1.0;
  double M[6] = {alpha, beta, (1 - alpha) * cx - beta * cy, -beta, alpha, beta * cx + (1 - alpha) * cy};
  double D = M[0] * M[4] - M[1] * M[3];
  D = D != 0 ? 1. / D : 0;
  const double A11 = M[4] * D, A22 = M[0] * D;
  M[0] = A11; M[1] *= -D; M[3] *= -D; M[4] = A22;
  const double b1 = -M[0] * M[2] - M[1] * M[5], b2 = -M[3] * M[2] - M[4] * M[5];
  M[2] = b1; M[5] = b2;
  auto rnd = [](double v) { return (int)std::nearbyint(v); };   // cvRound: half to even
  float tab1[32][2];
  for (int i = 0; i < 32; ++i) {
    const float x = i * (1.f / 32);
    tab1[i][0] = 1.f - x;
    tab1[i][1] = x;
  }
  for (int y = 0; y < k; ++y)
    for (int x = 0; x < k; ++x) {
      const int X0 = rnd((M[1] * y + M[2]) * 1024) + 16, Y0 = rnd((M[4] * y + M[5]) * 1024) + 16;
      const int X = (X0 + rnd(M[0] * x * 1024)) >> 5, Y = (Y0 + rnd(M[3] * x * 1024)) >> 5;
      const int sx = X >> 5, sy = Y >> 5, fx = X & 31, fy = Y & 31;
      const float w[4] = {tab1[fy][0] * tab1[fx][0], tab1[fy][0] * tab1[fx][1],
                          tab1[fy][1] * tab1[fx][0], tab1[fy][1] * tab1[fx][1]};
      auto src = [&](int xx, int yy) -> double {               // np.diag(np.ones(k)), 0 outside
        return xx >= 0 && yy >= 0 && xx < k && yy < k && xx == yy ? 1.0 : 0.0;
      };
      double v = 0.0;
      if (!(sx >= k || sx + 1 < 0 || sy >= k || sy + 1 < 0))
        v = src(sx, sy) * w[0] + src(sx + 1, sy) * w[1] + src(sx, sy + 1) * w[2] + src(sx + 1, sy + 1) * w[3];
      taps[y * RR_DISTORT_KMAX + x] = (float)(v / k);
    }
  for (int y = 0; y < RR_DISTORT_KMAX; ++y)
    for (int x = 0; x < RR_DISTORT_KMAX; ++x)
      if (y >= k || x >= k) taps[y * RR_DISTORT_KMAX + x] = 0.f;
  return RR_OK;
}

// all 11 x 361 motion-blur kernels of the draws above ([deg - 5][angle][KMAX^2])
extern "C" size_t rr_motion_blur_table_floats(void) {
  return (size_t)DRAW_NDEG * DRAW_NANG * RR_DISTORT_KMAX * RR_DISTORT_KMAX;
}

extern "C" int rr_motion_blur_table(float *table) {
  if (!table) return RR_EINVAL;
  for (int d = 0; d < DRAW_NDEG; ++d)
    for (int a = 0; a < DRAW_NANG; ++a) {
      const int rc = rr_motion_blur_kernel(DRAW_DEG0 + d, a,
                                           table + ((size_t)d * DRAW_NANG + a) * RR_DISTORT_KMAX * RR_DISTORT_KMAX);
      if (rc) return rc;
    }
  return RR_OK;
}

// workspace of rr_distort_random_u8: the blur staging image, the n draws, the
// n tap indices and the step's noise seed
static size_t draw_off_prm(int n, int h, int w, int c) {
  return ((size_t)n * h * w * c + 15) / 16 * 16;
}
extern "C" size_t rr_distort_random_workspace(int n, int h, int w, int c) {
  if (n <= 0 || h <= 0 || w <= 0 || c <= 0) return 0;
  return draw_off_prm(n, h, w, c) + (size_t)n * sizeof(rr_distort_param) + ((size_t)n * 4 + 15) / 16 * 16 + 16;
}

extern "C" int rr_distort_random_u8(int n, int h, int w, int c, const uint8_t *in, uint8_t *out,
                                    unsigned long long seed, long long *step, const float *table,
                                    void *ws, size_t ws_bytes, rr_stream stream) {
  if (!in || !out || !step || !table || !ws || n <= 0 || h <= 0 || w <= 0) return RR_EINVAL;
  if (c < 1 || c > 4) return RR_EINVAL;
  if (ws_bytes < rr_distort_random_workspace(n, h, w, c)) return RR_EWORKSPACE;
  char *base = (char *)ws;
  rr_distort_param *prm = (rr_distort_param *)(base + draw_off_prm(n, h, w, c));
  int *tap_idx = (int *)((char *)prm + (size_t)n * sizeof(rr_distort_param));
  unsigned long long *nseed = (unsigned long long *)((char *)tap_idx + ((size_t)n * 4 + 15) / 16 * 16);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(distort_draw_kernel, dim3(1), dim3(256), 0, st, n, seed, step, prm, tap_idx, nseed);
  RR_CHECK_LAUNCH();
  DistCfg a{n, h, w, c, 0, in, out, (uint8_t *)ws, prm, table, nullptr, 0ull, tap_idx, nseed};
  const long long te = (long long)n * h * w * c, tp = (long long)n * h * w;
  hipLaunchKernelGGL(distort_pre_kernel, dim3(rr_grid_cap((te + 255) / 256, 8192)), dim3(256), 0, st, a);
  RR_CHECK_LAUNCH();
  launch_blur(a, tp, st);
  RR_CHECK_LAUNCH();
  return RR_OK;
}

// the draws of the last rr_distort_random_u8 call, read back from its
// workspace (tests): params [n], tap indices [n], noise seed
extern "C" int rr_distort_random_draws(int n, int h, int w, int c, const void *ws,
                                       size_t *prm_off, size_t *idx_off, size_t *seed_off) {
  if (!ws || n <= 0 || !prm_off || !idx_off || !seed_off) return RR_EINVAL;
  *prm_off = draw_off_prm(n, h, w, c);
  *idx_off = *prm_off + (size_t)n * sizeof(rr_distort_param);
  *seed_off = *idx_off + ((size_t)n * 4 + 15) / 16 * 16;
  return RR_OK;
}
