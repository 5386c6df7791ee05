// common.h -- shared device helpers for the gfx950 kernels (CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/roadrestore.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef u16 u16x4 __attribute__((ext_vector_type(4)));
typedef u16 u16x8 __attribute__((ext_vector_type(8)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

// bf16 storage type: raw 16-bit pattern.
struct bf16_t {
  u16 v;
};

__device__ __forceinline__ float bf16_to_f32(u16 b) {
  return __uint_as_float(((uint32_t)b) << 16);
}
// round-to-nearest-even: the language conversion, which gfx950 lowers to
// v_cvt_pk_bf16_f32 (RNE, NaN stays NaN) -- no per-element branch
__device__ __forceinline__ u16 f32_to_bf16(float f) {
  return __builtin_bit_cast(u16, static_cast<__bf16>(f));
}

// Element traits: storage <-> fp32
template <typename T> struct Elt;
template <> struct Elt<float> {
  static constexpr int size = 4;
  static constexpr int dtype = RR_F32;
  __device__ __forceinline__ static float load(const float *p, long long i) { return p[i]; }
  __device__ __forceinline__ static void store(float *p, long long i, float v) { p[i] = v; }
  __device__ __forceinline__ static float round(float v) { return v; }   // (the stored value)
};
template <> struct Elt<bf16_t> {
  static constexpr int size = 2;
  static constexpr int dtype = RR_BF16;
  __device__ __forceinline__ static float load(const bf16_t *p, long long i) {
    return bf16_to_f32(p[i].v);
  }
  __device__ __forceinline__ static void store(bf16_t *p, long long i, float v) {
    p[i].v = f32_to_bf16(v);
  }
  __device__ __forceinline__ static float round(float v) { return bf16_to_f32(f32_to_bf16(v)); }
};

// 4 consecutive elements <-> float4
template <typename T> __device__ __forceinline__ f32x4 load4(const T *p);
template <> __device__ __forceinline__ f32x4 load4<float>(const float *p) {
  return *reinterpret_cast<const f32x4 *>(p);
}
template <> __device__ __forceinline__ f32x4 load4<bf16_t>(const bf16_t *p) {
  u16x4 r = *reinterpret_cast<const u16x4 *>(p);
  f32x4 o;
  o[0] = bf16_to_f32(r[0]); o[1] = bf16_to_f32(r[1]);
  o[2] = bf16_to_f32(r[2]); o[3] = bf16_to_f32(r[3]);
  return o;
}
template <typename T> __device__ __forceinline__ void store4(T *p, f32x4 v);
template <> __device__ __forceinline__ void store4<float>(float *p, f32x4 v) {
  *reinterpret_cast<f32x4 *>(p) = v;
}
template <> __device__ __forceinline__ void store4<bf16_t>(bf16_t *p, f32x4 v) {
  u16x4 r;
  r[0] = f32_to_bf16(v[0]); r[1] = f32_to_bf16(v[1]);
  r[2] = f32_to_bf16(v[2]); r[3] = f32_to_bf16(v[3]);
  *reinterpret_cast<u16x4 *>(p) = r;
}

// 8 consecutive elements (one 16-B bf16 store / two 16-B fp32 stores)
// 8 consecutive elements -> two f32x4 (one 16-B load for bf16)
template <typename T> __device__ __forceinline__ void load8(const T *p, f32x4 &a, f32x4 &b);
template <> __device__ __forceinline__ void load8<float>(const float *p, f32x4 &a, f32x4 &b) {
  a = *reinterpret_cast<const f32x4 *>(p);
  b = *reinterpret_cast<const f32x4 *>(p + 4);
}
template <> __device__ __forceinline__ void load8<bf16_t>(const bf16_t *p, f32x4 &a, f32x4 &b) {
  const uint4 r = *reinterpret_cast<const uint4 *>(p);
  a[0] = __uint_as_float(r.x << 16); a[1] = __uint_as_float(r.x & 0xffff0000u);
  a[2] = __uint_as_float(r.y << 16); a[3] = __uint_as_float(r.y & 0xffff0000u);
  b[0] = __uint_as_float(r.z << 16); b[1] = __uint_as_float(r.z & 0xffff0000u);
  b[2] = __uint_as_float(r.w << 16); b[3] = __uint_as_float(r.w & 0xffff0000u);
}

template <typename T> __device__ __forceinline__ void store8(T *p, f32x4 a, f32x4 b);
template <> __device__ __forceinline__ void store8<float>(float *p, f32x4 a, f32x4 b) {
  *reinterpret_cast<f32x4 *>(p) = a;
  *reinterpret_cast<f32x4 *>(p + 4) = b;
}
template <> __device__ __forceinline__ void store8<bf16_t>(bf16_t *p, f32x4 a, f32x4 b) {
  u16x8 r;
  r[0] = f32_to_bf16(a[0]); r[1] = f32_to_bf16(a[1]); r[2] = f32_to_bf16(a[2]); r[3] = f32_to_bf16(a[3]);
  r[4] = f32_to_bf16(b[0]); r[5] = f32_to_bf16(b[1]); r[6] = f32_to_bf16(b[2]); r[7] = f32_to_bf16(b[3]);
  *reinterpret_cast<u16x8 *>(p) = r;
}

// ---- reductions over the 16 lanes of a DPP row (lanes 16r .. 16r + 15) ----
// VALU data-parallel-primitive moves instead of __shfl_xor, which hipcc
// lowers to ds_bpermute_b32 (an LDS-pipe instruction with LDS latency: 368 of
// them in one conv3r epilogue).  The pairing follows the xor tree over lane
// offsets 1, 2, 4, 8: xor 1 and xor 2 are quad permutes; the last two steps
// pair each lane with one in the other quad of its 8 (row_half_mirror: 7 - i)
// and in the other half of the row (row_mirror: 15 - i).  After the first two
// steps every lane of a quad holds the quad's value, so the mirrors add the
// same operands as xor 4 / xor 8 would: the result is bitwise the xor tree's.
template <int CTRL> __device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<DPP_XOR1>(v);
  v += dpp_f<DPP_XOR2>(v);
  v += dpp_f<DPP_HALF_MIRROR>(v);
  v += dpp_f<DPP_MIRROR>(v);
  return v;
}
// max with the neighbouring lane (lane ^ 1)
__device__ __forceinline__ float max_xor1(float v) { return fmaxf(v, dpp_f<DPP_XOR1>(v)); }
// the neighbouring lane's (lane ^ 1) value, any 32-bit pattern
__device__ __forceinline__ uint32_t xor1_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_XOR1, 0xF, 0xF, false);
}
// MaxPool2d(2, 2) of one window in window order (0,0) (0,1) (1,0) (1,1):
// the value and the index of its FIRST occurrence (nn.MaxPool2d's routing of
// the backward), a NaN replacing a number (maxpool_fwd8_kernel's rule)
// take v over the running max m when v > m, or v is NaN and m is not:
// !(v <= m) is "v > m or either is NaN", and m == m excludes a NaN m -- the
// same truth table as (v > m || (v != v && m == m)) without the short-circuit,
// so it compiles to compares + v_cndmask instead of exec-mask branches (the
// branchy form cost ~14 instructions per window element in the pool
// epilogues)
__device__ __forceinline__ float pool4_first_max(float v0, float v1, float v2, float v3, uint32_t &id) {
  float m = v0;
  uint32_t k = 0;
  bool t = !(v1 <= m) & (m == m);
  m = t ? v1 : m; k = t ? 1u : k;
  t = !(v2 <= m) & (m == m);
  m = t ? v2 : m; k = t ? 2u : k;
  t = !(v3 <= m) & (m == m);
  m = t ? v3 : m; k = t ? 3u : k;
  id = k;
  return m;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

#define RR_CHECK_LAUNCH()                                   \
  do {                                                      \
    if (hipGetLastError() != hipSuccess) return RR_ELAUNCH; \
  } while (0)

// Kernel-path overrides for the parity tests, the library's one run-time
// knob: RR_PATH="key=value[,key=value...]" (read per call).  Every default is
// the measured-best path; the tests force a family off (conv3r=0,
// stream3=0, stream1=0, swgrad=0, igemm_halo=0, wgrad_halo=0, ...) or a
// workgroup kind (conv3r_wg=4/8, conv3r_segwg=4/8, conv3r_w64=0) to check
// one shipped kernel against another on the same shape.  Unknown keys are
// ignored; an unset variable costs one getenv.
static inline int rr_path(const char *key, int dflt) {
  const char *e = getenv("RR_PATH");
  if (!e || !*e) return dflt;
  const size_t kl = __builtin_strlen(key);
  for (const char *p = e; *p;) {
    const char *q = p;
    while (*q && *q != ',') ++q;
    const char *eq = p;
    while (eq < q && *eq != '=') ++eq;
    if (eq < q && (size_t)(eq - p) == kl && __builtin_memcmp(p, key, kl) == 0) return atoi(eq + 1);
    p = *q ? q + 1 : q;
  }
  return dflt;
}

static inline int rr_grid_cap(long long want, int cap = 2048) {
  if (want < 1) return 1;
  return (int)(want < cap ? want : cap);
}

// 256 zero bytes: out-of-bounds rows of an implicit-GEMM gather load from here.
static __device__ __attribute__((aligned(16))) const char rr_zero_page[256] = {0};

// Fast unsigned division by a runtime-invariant divisor (n < 2^31, d >= 1):
// q = (mulhi(n, m) + n) >> s with s = ceil(log2 d), m = floor(2^32 (2^s - d) / d) + 1.
struct FastDiv {
  uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv &f) {
  const uint32_t t = __umulhi(n, f.m);
  return (t + n) >> f.s;
}

// Fixed-order strided fp64 sums of NC interleaved components:
//   for (i = 0; i < n; ++i) s[k] += p[i * stride + k]
// with the loads of U iterations issued before their adds.  The add order is
// the plain loop's (bitwise-equal result); the plain loop compiles to one
// load -> wait -> add per iteration, i.e. one L2/HBM latency per row, which
// is what held the small finalize launches at 6-18 us.
template <int NC, int U = (NC == 1 ? 16 : 8), typename T>
__device__ __forceinline__ void rr_fixed_sum(const T *__restrict__ p, long long stride, long long n,
                                             double (&s)[NC]) {
  long long i = 0;
  for (; i + U <= n; i += U) {
    T v[U][NC];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < NC; ++k) v[u][k] = p[(i + u) * stride + k];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < NC; ++k) s[k] += (double)v[u][k];
  }
  for (; i < n; ++i)
#pragma unroll
    for (int k = 0; k < NC; ++k) s[k] += (double)p[i * stride + k];
}
// iterations of `for (i = first; i < end; i += step)`
__device__ __forceinline__ long long rr_trips(long long first, long long end, long long step) {
  return first < end ? (end - first + step - 1) / step : 0;
}

// Deterministic column reduction of fp32 partials: in [rows][cols] ->
// out [chunks][cols] in fp64 (fixed order).  grid (ceil(cols/64), chunks),
// 256 threads = 64 columns x 4 row lanes.  Feeds the finalize kernels so
// their sequential part is at most `chunks` rows.
__global__ static void rr_colreduce_kernel(const float *__restrict__ in, int rows, int cols,
                                           int rows_per_chunk, double *__restrict__ out) {
  __shared__ double red[4][64];
  const int tc = threadIdx.x & 63, l = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tc;
  const long long r0 = (long long)blockIdx.y * rows_per_chunk;
  const long long r1 = min((long long)rows, r0 + rows_per_chunk);
  double s[1] = {0.0};
  if (c < cols) rr_fixed_sum<1>(in + (r0 + l) * cols + c, 4LL * cols, rr_trips(r0 + l, r1, 4), s);
  red[l][tc] = s[0];
  __syncthreads();
  if (l == 0 && c < cols) out[(long long)blockIdx.y * cols + c] = red[0][tc] + red[1][tc] + red[2][tc] + red[3][tc];
}

static inline int rr_colreduce_chunks(int rows) { return rows < 64 ? (rows < 1 ? 1 : rows) : 64; }
static inline size_t rr_colreduce_bytes(int rows, int cols) {
  return (size_t)rr_colreduce_chunks(rows) * cols * sizeof(double);
}
static inline int rr_colreduce(const float *in, int rows, int cols, double *out, hipStream_t st) {
  const int chunks = rr_colreduce_chunks(rows);
  const int rpc = (rows + chunks - 1) / chunks;
  hipLaunchKernelGGL(rr_colreduce_kernel, dim3((cols + 63) / 64, chunks), dim3(256), 0, st, in, rows,
                     cols, rpc, out);
  return hipGetLastError() == hipSuccess ? chunks : -1;
}
