// Row-wise wavefront kernels: LayerNorm, 64-wide softmax, inverse L2 norm.
// One wave per row (or per 64-group); 4 rows per 256-thread workgroup; the
// whole row lives in registers, so every element is read from HBM once and
// reductions are 64-lane butterflies (no LDS).
#include "nr_common.h"

namespace nr {

// Lane-local load of 4 consecutive elements at element offset `e` (f32 or bf16).
template <typename T>
__device__ __forceinline__ void load4(const T* p, float (&v)[4]) {
  if constexpr (sizeof(T) == 4) {
    const float4 f = *reinterpret_cast<const float4*>(p);
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = bf16_lo(u.x); v[1] = bf16_hi(u.x); v[2] = bf16_lo(u.y); v[3] = bf16_hi(u.y);
  }
}

template <>
__device__ __forceinline__ void load4<_Float16>(const _Float16* p, float (&v)[4]) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4 h = *reinterpret_cast<const h4*>(p);
  v[0] = (float)h[0]; v[1] = (float)h[1]; v[2] = (float)h[2]; v[3] = (float)h[3];
}

template <typename T>
__device__ __forceinline__ void store4(T* p, const float (&v)[4]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    __bf16 b[4] = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    *reinterpret_cast<uint2*>(p) = *reinterpret_cast<uint2*>(b);
  }
}

// 16-byte lane vectors: E = 16 / sizeof(T) elements.
template <typename T>
__device__ __forceinline__ void load16(const T* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  if constexpr (sizeof(T) == 4) {
    v[0] = __uint_as_float(u.x); v[1] = __uint_as_float(u.y); v[2] = __uint_as_float(u.z); v[3] = __uint_as_float(u.w);
  } else {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) { v[2 * q] = bf16_lo(w[q]); v[2 * q + 1] = bf16_hi(w[q]); }
  }
}

template <typename TO, int E>
__device__ __forceinline__ void storeE(TO* p, const float* v) {
  if constexpr (sizeof(TO) == 4) {
#pragma unroll
    for (int q = 0; q < E; q += 4) *reinterpret_cast<float4*>(p + q) = make_float4(v[q], v[q + 1], v[q + 2], v[q + 3]);
  } else {
#pragma unroll
    for (int q = 0; q < E; q += 8) {
      __bf16 b8[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) b8[t] = (__bf16)v[q + t];
      *reinterpret_cast<uint4*>(p + q) = *reinterpret_cast<const uint4*>(b8);
    }
  }
}

// torch.nn.LayerNorm semantics: biased variance, y = (x - mean) * rsqrt(var + eps) * g + b.
// One wave per row, rows grid-strided over a bounded grid (tiny per-row work
// would otherwise be dispatch-bound); each lane holds 16-byte chunks, so a
// wave instruction moves 1 KiB; the whole row stays in registers.
template <typename TI, typename TO, int DIM>
__global__ __launch_bounds__(256) void layernorm_kernel(int64_t rows, const TI* __restrict__ x,
                                                        int64_t ldx, const float* __restrict__ g,
                                                        const float* __restrict__ b, float eps,
                                                        TO* __restrict__ y, int64_t ldy) {
  constexpr int E = 16 / (int)sizeof(TI);           // elements per lane chunk
  constexpr int CH = DIM / E;                        // chunks per row
  constexpr int NJ = (CH + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  // affine parameters of this lane's chunks, loaded once per wave
  float gv[NJ][E], bv[NJ][E];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = j * 64 + lane;
#pragma unroll
    for (int t = 0; t < E; ++t) {
      const bool ok = CH % 64 == 0 || c < CH;
      gv[j][t] = (g && ok) ? g[c * E + t] : 1.f;
      bv[j][t] = (b && ok) ? b[c * E + t] : 0.f;
    }
  }
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += nw) {
    float v[NJ][E];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = j * 64 + lane;
      if (CH % 64 == 0 || c < CH) {
        load16<TI>(x + row * ldx + c * E, v[j]);
#pragma unroll
        for (int t = 0; t < E; ++t) s += v[j][t];
      }
    }
    const float mean = wave_sum(s) / (float)DIM;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = j * 64 + lane;
      if (CH % 64 == 0 || c < CH) {
#pragma unroll
        for (int t = 0; t < E; ++t) {
          const float d = v[j][t] - mean;
          q = fmaf(d, d, q);
        }
      }
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)DIM + eps);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = j * 64 + lane;
      if (CH % 64 == 0 || c < CH) {
        float o[E];
#pragma unroll
        for (int t = 0; t < E; ++t) o[t] = (v[j][t] - mean) * rstd * gv[j][t] + bv[j][t];
        storeE<TO, E>(y + row * ldy + c * E, o);
      }
    }
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void softmax64_kernel(int64_t items, int64_t groups,
                                                        const float* __restrict__ x, int64_t ldx,
                                                        TO* __restrict__ y, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (it >= items) return;
  const int64_t row = it / groups, grp = it % groups;
  const float v = x[row * ldx + grp * 64 + lane];
  const float m = wave_max(v);
  const float e = expf(v - m);
  const float s = wave_sum(e);
  const float o = e / s;
  if constexpr (sizeof(TO) == 4) y[row * ldy + grp * 64 + lane] = o;
  else y[row * ldy + grp * 64 + lane] = (TO)o;
}

// Per-row LayerNorm statistics (mean, rstd) with the LayerNorm kernel's exact
// arithmetic (two passes over the register-resident row, biased variance):
// the bf16 latent transform applies LN inside the next GEMM's epilogue
// (gemm256t_kernel LNF) instead of writing the normalised rows.
template <typename T, int DIM>
__global__ __launch_bounds__(256) void row_stats_kernel(int64_t rows, const T* __restrict__ x, int64_t ldx,
                                                        float eps, float2* __restrict__ out) {
  constexpr int E = 16 / (int)sizeof(T);
  constexpr int NJ = DIM / (64 * E);
  static_assert(DIM % (64 * E) == 0, "row_stats: DIM must be a multiple of 64 lanes x 16 B");
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += nw) {
    float v[NJ][E];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      load16<T>(x + row * ldx + (j * 64 + lane) * E, v[j]);
#pragma unroll
      for (int t = 0; t < E; ++t) s += v[j][t];
    }
    const float mean = wave_sum(s) / (float)DIM;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int t = 0; t < E; ++t) {
        const float d = v[j][t] - mean;
        q = fmaf(d, d, q);
      }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)DIM + eps);
    if (lane == 0) out[row] = make_float2(mean, rstd);
  }
}

template <typename T, int DIM>
__global__ __launch_bounds__(256) void inv_norm_kernel(int64_t rows, const T* __restrict__ x,
                                                       int64_t ldx, float eps,
                                                       float* __restrict__ out) {
  constexpr int NJ = DIM / 256;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    float v[4];
    load4<T>(x + row * ldx + j * 256 + lane * 4, v);
#pragma unroll
    for (int t = 0; t < 4; ++t) q = fmaf(v[t], v[t], q);
  }
  q = wave_sum(q);
  if (lane == 0) out[row] = 1.0f / fmaxf(sqrtf(q), eps);
}

template <typename TI, typename TO>
static int launch_ln(int64_t rows, int64_t dim, const void* x, int64_t ldx, const float* g,
                     const float* b, float eps, void* y, int64_t ldy, hipStream_t s) {
  const int64_t nb = (rows + 3) / 4;
  constexpr int64_t cap = 1024;  // grid cap (measured best for bf16 at 72k rows)
  const dim3 grid((unsigned)(cap > 0 && nb > cap ? cap : nb));  // rows grid-strided over <= cap blocks
#define NR_LN_CASE(D)                                                                      \
  case D:                                                                                  \
    hipLaunchKernelGGL((layernorm_kernel<TI, TO, D>), grid, dim3(256), 0, s, rows,        \
                       (const TI*)x, ldx, g, b, eps, (TO*)y, ldy);                          \
    break;
  switch (dim) {
    NR_LN_CASE(256) NR_LN_CASE(512) NR_LN_CASE(768) NR_LN_CASE(1024) NR_LN_CASE(2048)
    default: set_error("nr_layernorm: dim %lld unsupported", (long long)dim); return NR_ERR_UNSUPPORTED;
  }
#undef NR_LN_CASE
  NR_CHECK_LAUNCH("nr_layernorm");
  return NR_OK;
}

int layernorm_dispatch(int dti, int dto, int64_t rows, int64_t dim, const void* x, int64_t ldx,
                       const float* g, const float* b, float eps, void* y, int64_t ldy,
                       hipStream_t s) {
  NR_CHECK_ARG((dti == NR_F32 || dti == NR_BF16) && (dto == NR_F32 || dto == NR_BF16), "nr_layernorm: bad dtype");
  NR_CHECK_ARG(rows >= 0 && ldx >= dim && ldy >= dim, "nr_layernorm: bad strides");
  NR_CHECK_ARG((ldx * (dti == NR_F32 ? 4 : 2)) % 16 == 0 && (ldy * (dto == NR_F32 ? 4 : 2)) % 16 == 0 &&
                   ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0,
               "nr_layernorm: rows must be 16-byte aligned");
  if (rows == 0) return NR_OK;
  NR_CHECK_ARG(x && y, "nr_layernorm: null pointer");
  if (dti == NR_F32) {
    if (dto == NR_F32) return launch_ln<float, float>(rows, dim, x, ldx, g, b, eps, y, ldy, s);
    return launch_ln<float, __bf16>(rows, dim, x, ldx, g, b, eps, y, ldy, s);
  }
  if (dto == NR_F32) return launch_ln<__bf16, float>(rows, dim, x, ldx, g, b, eps, y, ldy, s);
  return launch_ln<__bf16, __bf16>(rows, dim, x, ldx, g, b, eps, y, ldy, s);
}

int softmax64_dispatch(int64_t rows, int64_t groups, const float* x, int64_t ldx, int dto, void* y,
                       int64_t ldy, hipStream_t s) {
  NR_CHECK_ARG(rows >= 0 && groups > 0 && ldx >= groups * 64 && ldy >= groups * 64, "nr_softmax64: bad shape");
  NR_CHECK_ARG(dto == NR_F32 || dto == NR_BF16, "nr_softmax64: bad dtype");
  if (rows == 0) return NR_OK;
  NR_CHECK_ARG(x && y, "nr_softmax64: null pointer");
  const int64_t items = rows * groups;
  const dim3 grid((unsigned)((items + 3) / 4));
  if (dto == NR_F32)
    hipLaunchKernelGGL((softmax64_kernel<float>), grid, dim3(256), 0, s, items, groups, x, ldx, (float*)y, ldy);
  else
    hipLaunchKernelGGL((softmax64_kernel<__bf16>), grid, dim3(256), 0, s, items, groups, x, ldx, (__bf16*)y, ldy);
  NR_CHECK_LAUNCH("nr_softmax64");
  return NR_OK;
}

int inv_norm_dispatch(int dtype, int64_t rows, int64_t dim, const void* x, int64_t ldx, float eps,
                      float* out, hipStream_t s) {
  NR_CHECK_ARG(dtype == NR_F32 || dtype == NR_BF16, "nr_row_inv_norm: bad dtype");
  NR_CHECK_ARG(rows >= 0 && ldx >= dim && ldx % 4 == 0, "nr_row_inv_norm: bad strides");
  if (rows == 0) return NR_OK;
  NR_CHECK_ARG(x && out, "nr_row_inv_norm: null pointer");
  const dim3 grid((unsigned)((rows + 3) / 4));
#define NR_IN_CASE(T, D)                                                                        \
  case D:                                                                                       \
    hipLaunchKernelGGL((inv_norm_kernel<T, D>), grid, dim3(256), 0, s, rows, (const T*)x, ldx,  \
                       eps, out);                                                               \
    break;
  if (dtype == NR_F32) {
    switch (dim) {
      NR_IN_CASE(float, 256) NR_IN_CASE(float, 512) NR_IN_CASE(float, 768) NR_IN_CASE(float, 1024) NR_IN_CASE(float, 2048)
      default: set_error("nr_row_inv_norm: dim %lld unsupported", (long long)dim); return NR_ERR_UNSUPPORTED;
    }
  } else {
    switch (dim) {
      NR_IN_CASE(__bf16, 256) NR_IN_CASE(__bf16, 512) NR_IN_CASE(__bf16, 768) NR_IN_CASE(__bf16, 1024) NR_IN_CASE(__bf16, 2048)
      default: set_error("nr_row_inv_norm: dim %lld unsupported", (long long)dim); return NR_ERR_UNSUPPORTED;
    }
  }
#undef NR_IN_CASE
  NR_CHECK_LAUNCH("nr_row_inv_norm");
  return NR_OK;
}


// Gathered chain of LayerNorms: out[i] = LN_{n-1}(...LN_0(x[row_idx[i]])...),
// f32 math and output.  The token-attention encoder's effective forward
// (attention.py:174-194 returns g_mlp_layernorm(hidden_states); the attention
// branch is dead) followed by last_token_pool (modeling_utils.py:37-48) is one
// such LN of the last valid token row, so only those rows are ever read.
template <typename TI, int DIM>
__global__ __launch_bounds__(256) void gather_ln_kernel(int64_t n, const TI* __restrict__ x, int64_t ldx,
                                                        const int64_t* __restrict__ row_idx, int n_ln,
                                                        const float* __restrict__ g, const float* __restrict__ b,
                                                        float eps, float* __restrict__ y, int64_t ldy) {
  constexpr int NJ = DIM / 256;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t row = row_idx ? row_idx[i] : i;
  float v[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j) load4<TI>(x + row * ldx + j * 256 + lane * 4, v[j]);
  for (int l = 0; l < n_ln; ++l) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
    const float mean = wave_sum(s) / (float)DIM;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float d = v[j][t] - mean;
        q = fmaf(d, d, q);
      }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)DIM + eps);
    const float* gl = g ? g + (int64_t)l * DIM : nullptr;
    const float* bl = b ? b + (int64_t)l * DIM : nullptr;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int e = j * 256 + lane * 4 + t;
        v[j][t] = (v[j][t] - mean) * rstd * (gl ? gl[e] : 1.f) + (bl ? bl[e] : 0.f);
      }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) store4<float>(y + i * ldy + j * 256 + lane * 4, v[j]);
}

int gather_ln_dispatch(int dti, int64_t n, int64_t dim, const void* x, int64_t ldx, const int64_t* row_idx,
                       int n_ln, const float* g, const float* b, float eps, float* y, int64_t ldy,
                       hipStream_t s) {
  NR_CHECK_ARG(dti == NR_F32 || dti == NR_BF16 || dti == NR_F16, "nr_gather_layernorm: bad dtype");
  NR_CHECK_ARG(n >= 0 && n_ln >= 0 && ldx >= dim && ldy >= dim && ldx % 4 == 0 && ldy % 4 == 0,
               "nr_gather_layernorm: bad shape/strides");
  if (n == 0) return NR_OK;
  NR_CHECK_ARG(x && y, "nr_gather_layernorm: null pointer");
  NR_CHECK_ARG(dim == 1024 || dim == 512 || dim == 2048 || dim == 256, "nr_gather_layernorm: dim %lld unsupported",
               (long long)dim);
  const dim3 grid((unsigned)((n + 3) / 4));
#define NR_GL(T, D)                                                                                   \
  if (dim == D) {                                                                                     \
    hipLaunchKernelGGL((gather_ln_kernel<T, D>), grid, dim3(256), 0, s, n, (const T*)x, ldx, row_idx, \
                       n_ln, g, b, eps, y, ldy);                                                      \
  }
#define NR_GL_ALL(T) NR_GL(T, 256) NR_GL(T, 512) NR_GL(T, 1024) NR_GL(T, 2048)
  if (dti == NR_F32) { NR_GL_ALL(float) }
  else if (dti == NR_BF16) { NR_GL_ALL(__bf16) }
  else { NR_GL_ALL(_Float16) }
#undef NR_GL_ALL
#undef NR_GL
  NR_CHECK_LAUNCH("nr_gather_layernorm");
  return NR_OK;
}

int row_stats_dispatch(int dtype, int64_t rows, int64_t dim, const void* x, int64_t ldx, float eps, float* out,
                       hipStream_t s) {
  NR_CHECK_ARG(dtype == NR_F32 || dtype == NR_BF16, "nr_row_stats: bad dtype");
  NR_CHECK_ARG(dim == 1024, "nr_row_stats: dim %lld unsupported (1024 only)", (long long)dim);
  NR_CHECK_ARG(rows >= 0 && ldx >= dim && (ldx * (dtype == NR_F32 ? 4 : 2)) % 16 == 0 && ((uintptr_t)x & 15) == 0 &&
                   ((uintptr_t)out & 7) == 0,
               "nr_row_stats: rows must be 16-byte aligned, out 8-byte aligned");
  if (rows == 0) return NR_OK;
  NR_CHECK_ARG(x && out, "nr_row_stats: null pointer");
  const int64_t nb = (rows + 3) / 4;
  const dim3 grid((unsigned)(nb > 2048 ? 2048 : nb));
  if (dtype == NR_F32)
    hipLaunchKernelGGL((row_stats_kernel<float, 1024>), grid, dim3(256), 0, s, rows, (const float*)x, ldx, eps,
                       (float2*)out);
  else
    hipLaunchKernelGGL((row_stats_kernel<__bf16, 1024>), grid, dim3(256), 0, s, rows, (const __bf16*)x, ldx, eps,
                       (float2*)out);
  NR_CHECK_LAUNCH("nr_row_stats");
  return NR_OK;
}

}  // namespace nr

extern "C" int nr_gather_layernorm(int dtype_in, int64_t n, int64_t dim, const void* x, int64_t ldx,
                                   const int64_t* row_idx, int n_ln, const float* gammas, const float* betas,
                                   float eps, float* out, int64_t ldo, void* stream) {
  nr::clear_error();
  if (n > 0) NR_CHECK_DEVICE("nr_gather_layernorm", x, row_idx, gammas, betas, out);
  return nr::gather_ln_dispatch(dtype_in, n, dim, x, ldx, row_idx, n_ln, gammas, betas, eps, out, ldo,
                                (hipStream_t)stream);
}

extern "C" int nr_layernorm(int dtype_in, int dtype_out, int64_t rows, int64_t dim, const void* x,
                            int64_t ldx, const float* gamma, const float* beta, float eps, void* y,
                            int64_t ldy, void* stream) {
  nr::clear_error();
  if (rows > 0) NR_CHECK_DEVICE("nr_layernorm", x, gamma, beta, y);
  return nr::layernorm_dispatch(dtype_in, dtype_out, rows, dim, x, ldx, gamma, beta, eps, y, ldy,
                                (hipStream_t)stream);
}

extern "C" int nr_softmax64(int64_t rows, int64_t groups, const float* x, int64_t ldx,
                            int dtype_out, void* y, int64_t ldy, void* stream) {
  nr::clear_error();
  if (rows > 0) NR_CHECK_DEVICE("nr_softmax64", x, y);
  return nr::softmax64_dispatch(rows, groups, x, ldx, dtype_out, y, ldy, (hipStream_t)stream);
}

extern "C" int nr_row_inv_norm(int dtype, int64_t rows, int64_t dim, const void* x, int64_t ldx,
                               float eps, float* out, void* stream) {
  nr::clear_error();
  if (rows > 0) NR_CHECK_DEVICE("nr_row_inv_norm", x, out);
  return nr::inv_norm_dispatch(dtype, rows, dim, x, ldx, eps, out, (hipStream_t)stream);
}

extern "C" int nr_row_stats(int dtype, int64_t rows, int64_t dim, const void* x, int64_t ldx, float eps, float* out,
                            void* stream) {
  nr::clear_error();
  if (rows > 0) NR_CHECK_DEVICE("nr_row_stats", x, out);
  return nr::row_stats_dispatch(dtype, rows, dim, x, ldx, eps, out, (hipStream_t)stream);
}
