// Shared helpers for the newsrec HIP library (gfx950 / CDNA4 only).
//
// Error model of the C-ABI (include/newsrec.h): every entry point returns
// NR_OK (0) or a negative code; the message is kept in a thread-local buffer
// readable through nr_last_error().  No C++ exception crosses the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include <initializer_list>

#include "../../include/newsrec.h"

namespace nr {

void set_error(const char* fmt, ...);
void clear_error();

// Device residency of caller pointers (capi.hip): true for device / managed
// memory.  check_device_ptrs names the first offending argument of the
// stringified list `names`; null pointers are skipped (nullable arguments).
bool device_accessible(const void* p);
void residency_flush();  // drop every thread's verified ranges (nr_residency_flush)
int check_device_ptrs(const char* fn, const char* names, std::initializer_list<const void*> ptrs);

// internal dispatchers (validate + launch, no error reset)
int gemm_dispatch(int dtype_in, int dtype_out, int epi, int64_t M, int64_t N, int64_t K,
                  const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
                  const void* R, int64_t ldr, void* C, int64_t ldc, hipStream_t s);
// Extra epilogue arguments of the GEMMs (gemm.hip): dropout of the training
// forward, the LayerNorm fold, the persistent kernel's column sums.
struct EpiArgs {
  uint64_t seed;  // dropout stream
  uint32_t thr;   // drop iff drop_at(seed, row * N + col, thr)  (thr = round(p * 2^16), dropout_threshold)
  float scale;    // 1 / (1 - p)
  int group_m = 1;  // 256x256 tile order: >1 groups group_m M-tiles (see tile_of)
  const float* ln_stats = nullptr;  // LNF epilogue: [M] (mean, rstd) pairs
  const float* ln_uc = nullptr;     // LNF epilogue: u [N] then c [N]
  float* colsum = nullptr;          // persistent kernel, CS: [ceil(M / 128)][N] f32 column sums of each 128-row block
  float* sq_part = nullptr;         // 256x256 tile kernels: per-workgroup sum of squares of the stored values
  bool sq_on = false;               //   (written at sq_part[blockIdx.x]; 0 when !sq_on)
};

int gemm_dispatch_ex(int dtype_in, int dtype_out, int epi, int64_t M, int64_t N, int64_t K,
                     const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
                     const void* R, int64_t ldr, void* C, int64_t ldc, const EpiArgs& ea, hipStream_t s);
int layernorm_dispatch(int dti, int dto, int64_t rows, int64_t dim, const void* x, int64_t ldx,
                       const float* g, const float* b, float eps, void* y, int64_t ldy,
                       hipStream_t s);
int softmax64_dispatch(int64_t rows, int64_t groups, const float* x, int64_t ldx, int dto, void* y,
                       int64_t ldy, hipStream_t s);
int gather_ln_dispatch(int dti, int64_t n, int64_t dim, const void* x, int64_t ldx, const int64_t* row_idx,
                       int n_ln, const float* g, const float* b, float eps, float* y, int64_t ldy, hipStream_t s);
int pool_rows_dispatch(int pooler, int dtype, const void* table, int64_t ld, const int64_t* off, int64_t n_seg,
                       float* users, hipStream_t s);
int row_stats_dispatch(int dtype, int64_t rows, int64_t dim, const void* x, int64_t ldx, float eps, float* out,
                       hipStream_t s);
// bf16 persistent GEMM with a LayerNorm folded into its epilogue (epi NR_EPI_SOFTMAX64 or
// NR_EPI_GEGLU): C = epi(rstd_m * (A W^T - mean_m u_n) + c_n); stats [M] (mean, rstd), uc [2][N]
int gemm_lnfold_dispatch(int epi, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* W,
                         int64_t ldw, const float* stats, const float* uc, void* C, int64_t ldc, hipStream_t s);
// The training steps' side streams (latent_train.hip): two non-blocking streams
// and their fork / join events per host thread and device, created on first use
// on the DEVICE OF `st` (not the caller's current device) and kept.
struct TrainSide {
  hipStream_t s = nullptr, s2 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr, fork2 = nullptr, join2 = nullptr, wt = nullptr;
};
int train_side_streams(hipStream_t st, const char* fn, TrainSide& out);

// One problem of a grouped GEMM launch (gemm.hip gemm_group_dispatch): C = alpha A W^T,
// no bias; `batch` instances at A + b sA, W + b sW, C + b sC (element strides).
struct GemmProblem {
  int64_t M, N, K;
  const void* A;
  int64_t lda, sA;
  const void* W;
  int64_t ldw, sW;
  void* C;
  int64_t ldc, sC;
  int batch;
  float alpha;
};
constexpr int kGroupMax = 16;
// sq_part (nullable): per-workgroup sums of squares of the problems flagged in sq (0 for
// the others), one per workgroup; refused before launch when the workgroup count
// exceeds sq_cap; *n_tiles (nullable) = the workgroup count.
int gemm_group_dispatch(int dtype_in, int dtype_out, const GemmProblem* probs, int n, hipStream_t s,
                        float* sq_part = nullptr, const bool* sq = nullptr, int* n_tiles = nullptr,
                        int sq_cap = 0);
// C = alpha A^T W per problem, A [K][M] and W [K][N] bf16 row-major (gemm.hip, TN grouped launch)
// sq_part (nullable): per-workgroup sums of squares of the problems flagged in sq
// (0 for the others), one per workgroup, refused before launch past sq_cap workgroups;
// *n_tiles (nullable) = the workgroup count.
int gemm_group_tn_dispatch(int dtype_out, const GemmProblem* probs, int n, hipStream_t s, float* sq_part = nullptr,
                           const bool* sq = nullptr, int* n_tiles = nullptr, int sq_cap = 0);
int inv_norm_dispatch(int dtype, int64_t rows, int64_t dim, const void* x, int64_t ldx, float eps,
                      float* out, hipStream_t s);

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// Counter-based dropout stream: one splitmix64 finaliser output of seed + (g+1) *
// golden ratio per group g of 4 consecutive elements of a row (element idx = row
// * N + col, N % 4 == 0, is in group idx >> 2); element idx is dropped iff the
// 16-bit field idx & 3 of its group's hash is < thr = round(p * 2^16).  (One
// hash per 4 elements: the RELU_DROPOUT epilogues spent more time in per-element
// 64-bit hashes than in the ReLU GEMM's epilogue itself.)  oracle/train_ref.py
// restates it in numpy so the CPU checker draws exactly the same masks.
__device__ __forceinline__ uint64_t drop_hash4(uint64_t seed, uint64_t g) {
  uint64_t z = seed + (g + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ bool drop_field(uint64_t h, int k, uint32_t thr) {
  return ((uint32_t)(h >> (16 * k)) & 0xffffu) < thr;
}
// host: the 16-bit drop threshold of probability p (p quantised to 1/65536; the
// keep scale stays 1 / (1 - p))
static inline uint32_t dropout_threshold(float p) {
  const double t = __builtin_nearbyint((double)p * 65536.0);
  return t <= 0.0 ? 0u : t >= 65536.0 ? 65536u : (uint32_t)t;
}
// the per-element form (tile kernels): element idx of the stream
__device__ __forceinline__ bool drop_at(uint64_t seed, uint64_t idx, uint32_t thr) {
  return drop_field(drop_hash4(seed, idx >> 2), (int)(idx & 3), thr);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// GELU of four values (two float2 chains, v_pk_fma_f32 / v_pk_mul_f32) for the
// persistent bf16 kernel's GELU and GEGLU epilogues (gemm.hip) and the
// latent step's bf16 GEGLU (latent_train.hip).  Round 4: no reciprocal.
// With s = g sqrt(log2(e) / 2) (so s^2 = log2(e) z^2, z = |g| / sqrt 2),
//   erfc(z) = 2^(P(min(|s|, 4 sqrt(log2 e))) - s^2),
// P(s) ~ log2(erfcx(s / sqrt(log2 e))) a degree-8 polynomial (Lawson minimax on
// z in [0, 4]: |error| <= 3.2e-6 in log2 units, 2.2e-6 relative on erfc; past
// z = 4 only erfc's Gaussian factor keeps falling, where gelu is g or ~0 to
// 1e-8).  gelu = g (1 - erfc / 2) for g >= 0, g erfc / 2 below: |gelu - exact|
// <= 3.9e-7 over |g| <= 12 in f32, as the Numerical-Recipes erfc form of
// gelu_erf (3.8e-7) -- checked in float64 emulation of these f32 steps.  Per
// four values 2 fewer pk_fma chains steps, no v_rcp_f32 and no t multiply:
// the plain-GELU epilogue (encoder FFN1) cost 22 % of its GEMM at the ff1
// shape (probe 0.961 -> 1.171 ms, profiles/round4/gemm/r4g5_*).  The f32
// kernels keep gelu_erf.
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2v fma2(f32x2v a, f32x2v b, f32x2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ void gelu_erf2x2(f32x2v& g0, f32x2v& g1) {
  constexpr float kS = 0.8493218002880191f, kSmax = 4.804489635145799f;
  const f32x2v s0 = g0 * kS, s1 = g1 * kS;
  const f32x2v c0 = {fminf(fabsf(s0.x), kSmax), fminf(fabsf(s0.y), kSmax)};
  const f32x2v c1 = {fminf(fabsf(s1.x), kSmax), fminf(fabsf(s1.y), kSmax)};
  f32x2v p0 = (f32x2v)-3.57632359e-07f, p1 = (f32x2v)-3.57632359e-07f;
#define NR_G4(c)                      \
  p0 = fma2(p0, c0, (f32x2v)(c)); \
  p1 = fma2(p1, c1, (f32x2v)(c));
  NR_G4(8.19052786e-07f) NR_G4(0.000115395807f) NR_G4(-0.00191940868f) NR_G4(0.0159611721f)
  NR_G4(-0.0876397938f) NR_G4(0.364198327f) NR_G4(-1.35544741f) NR_G4(3.20236495e-06f - 1.0f)
#undef NR_G4
  // w = P - 1 - s^2: 2^w = erfc / 2; gelu = max(g, 0) - |g| erfc / 2 (g (1 - erfc / 2)
  // for g >= 0, g erfc / 2 below) -- one fma with |.| / neg modifiers, no select
  const f32x2v w0 = fma2(-s0, s0, p0), w1 = fma2(-s1, s1, p1);
  // max(g, 0) as a signed-integer max on the bits (a negative float, -0 included,
  // is a negative int): one v_max_i32, where fmaxf adds an IEEE canonicalize
  auto relu = [](float v) { return __int_as_float(max(__float_as_int(v), 0)); };
  g0 = (f32x2v){fmaf(-fabsf(g0.x), __builtin_amdgcn_exp2f(w0.x), relu(g0.x)),
                fmaf(-fabsf(g0.y), __builtin_amdgcn_exp2f(w0.y), relu(g0.y))};
  g1 = (f32x2v){fmaf(-fabsf(g1.x), __builtin_amdgcn_exp2f(w1.x), relu(g1.x)),
                fmaf(-fabsf(g1.y), __builtin_amdgcn_exp2f(w1.y), relu(g1.y))};
}

}  // namespace nr

#define NR_CHECK_ARG(cond, ...)                 \
  do {                                          \
    if (!(cond)) {                              \
      nr::set_error(__VA_ARGS__);               \
      return NR_ERR_INVALID;                    \
    }                                           \
  } while (0)

// Every public entry validates the pointers it hands to a kernel:
//   NR_CHECK_DEVICE("nr_pool_score", hist_table, cand_table, ...);
#define NR_CHECK_DEVICE(fn, ...)                                                 \
  do {                                                                           \
    const int _rc = nr::check_device_ptrs(fn, #__VA_ARGS__, {__VA_ARGS__});      \
    if (_rc) return _rc;                                                         \
  } while (0)

#define NR_CHECK_LAUNCH(name)                                               \
  do {                                                                        \
    hipError_t _e = hipGetLastError();                                        \
    if (_e != hipSuccess) {                                                   \
      nr::set_error("%s: launch failed: %s", name, hipGetErrorString(_e));    \
      return NR_ERR_HIP;                                                      \
    }                                                                         \
  } while (0)
