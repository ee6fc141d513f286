// Config-5 training step with the latent pooler (BASELINE configs[4]: "bf16
// MFMA backward for encoder + latent attention"), forward and backward of one
// batch as one C call (nr_latent_train_step, include/newsrec.h).  The math is
// the reference trainer's loop body (trainer.py:1044-1066) with
// LatentAttentionModel (latent_attention.py:134-171) in FinalAttention's slot:
//
//   E  = g_mlp_LN(last token)                        token model (attention.py:193)
//        (never stored as a [U][1024] table: the slot gather, the head's pos / neg
//        rows and the LN_q backward recompute E rows from the token states, tok_ln)
//   fold (weights only, once per step; the reference rebuilds K/V per batch row,
//   latent_attention.py:161-162):
//        KV = LN_c(latents) Wkv^T;  A_h = K_h Wq_h / sqrt(512);  BtT_h = V_h Wo_h^T
//   per history slot (packed valid rows, CSR order, zero rows up to Hp = pad64(Hs)):
//        S = E[hist];  X = LN_q(S);  P = softmax64(X A^T);  H1 = P Bt^T + S
//        G = LN_f(H1) W1^T + b1;  Z = a * gelu(g), (a, g) = G.chunk(2)
//   per batch row b (h_b slots):
//        m_b = mean(Z) W2^T + b2 + mean(H1)  ==  mean(Z W2^T + b2 + H1) = mean(H)
//        u_b = normalize(m_b);  loss = mean(max(0, 2 - cos(u, E[pos]) + cos(u, E[neg])))
// The last linear layer commutes with the history mean, so its forward GEMM,
// its data-grad GEMM and its weight-grad GEMM run over B rows instead of Hs
// slots (exact up to f32 summation order; the reference computes H per padded
// slot).  Backward:
//   dm (normalize backward) -> dZ_b = (dm_b / h_b) W2 (per row, broadcast to its
//   slots) -> dG = GEGLU' -> dY = dG W1 -> dH1 = LN_f'(dY) + dm_b / h_b ->
//   dP = dH1 Bt -> dS = softmax64'(P, dP) -> dX = dS A -> dE_slot = LN_q'(dX) + dH1,
//   and the token LN's parameter grads straight from the slots' dE_slot and the pos /
//   neg rows' cosine grads (linear in dE: no [U][1024] dE table is formed)
//   weight grads: W1 = dG^T Y, W2 = dm^T mean(Z), A = dS^T X, Bt = dH1^T P (one
//   grouped launch), then the fold backward (Wq, Wkv, Wo, latents, norm_context)
//   as two grouped launches of the 8 heads, and the LN parameter grads.
// GEMMs: nr's MFMA kernels (gemm.hip: persistent bf16, grouped strided batches);
// everything else here is HBM-bound row work (one wave per row, 16-B lanes).
#include "nr_common.h"

namespace nr {
namespace lt {

constexpr int D = 1024, F = 4096, S = 512, NL = 64, HEADS = 8, DH = 512;

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float v[4]) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = bf16_lo(u.x); v[1] = bf16_hi(u.x); v[2] = bf16_lo(u.y); v[3] = bf16_hi(u.y);
  }
}

__device__ __forceinline__ uint32_t pk2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{a, b}, b2));
}

template <typename T>
__device__ __forceinline__ void st4(T* p, const float v[4]) {
  if constexpr (sizeof(T) == 4) *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
  else *reinterpret_cast<uint2*>(p) = uint2{pk2(v[0], v[1]), pk2(v[2], v[3])};
}

template <typename T>
__device__ __forceinline__ void st4z(T* p) {
  const float z[4] = {0.f, 0.f, 0.f, 0.f};
  st4<T>(p, z);
}

__device__ __forceinline__ float gelu_x(float g) { return 0.5f * g * (1.0f + erff(g * 0.70710678118654752440f)); }

// bf16 step only (the f32 step keeps erff / expf): for two values, h = erfc(|g| /
// sqrt 2) / 2 and e = exp(-g^2 / 2) with one packed polynomial and v_exp_f32, no
// branches -- the erfc form of gelu_erf2x2 (nr_common.h: s = g sqrt(log2(e) / 2),
// erfc = 2^(P(min(|s|, 4 sqrt(log2 e))) - s^2), P a degree-8 minimax fit of
// log2(erfcx), its -1 folded in so 2^(P - s^2) = erfc / 2; relative error <= 2.2e-6
// on erfc).  The divergent two-range erff plus expf made GEGLU's backward
// VALU-heavy (~65 instructions per element).
__device__ __forceinline__ void erfc_half2(f32x2v g, f32x2v& h, f32x2v& e) {
  constexpr float kS = 0.8493218002880191f, kSmax = 4.804489635145799f;
  const f32x2v s = g * kS;
  const f32x2v c = {fminf(fabsf(s.x), kSmax), fminf(fabsf(s.y), kSmax)};
  f32x2v q = (f32x2v)-3.57632359e-07f;
  q = fma2(q, c, (f32x2v)8.19052786e-07f);
  q = fma2(q, c, (f32x2v)0.000115395807f);
  q = fma2(q, c, (f32x2v)-0.00191940868f);
  q = fma2(q, c, (f32x2v)0.0159611721f);
  q = fma2(q, c, (f32x2v)-0.0876397938f);
  q = fma2(q, c, (f32x2v)0.364198327f);
  q = fma2(q, c, (f32x2v)-1.35544741f);
  q = fma2(q, c, (f32x2v)(3.20236495e-06f - 1.0f));
  const f32x2v ns2 = -s * s, w = q + ns2;
  e = (f32x2v){__builtin_amdgcn_exp2f(ns2.x), __builtin_amdgcn_exp2f(ns2.y)};
  h = (f32x2v){__builtin_amdgcn_exp2f(w.x), __builtin_amdgcn_exp2f(w.y)};
}

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float v[8]) {
  if constexpr (sizeof(T) == 4) {
    ld4<float>(p, v);
    ld4<float>(p + 4, v + 4);
  } else {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    v[0] = bf16_lo(u.x); v[1] = bf16_hi(u.x); v[2] = bf16_lo(u.y); v[3] = bf16_hi(u.y);
    v[4] = bf16_lo(u.z); v[5] = bf16_hi(u.z); v[6] = bf16_lo(u.w); v[7] = bf16_hi(u.w);
  }
}

template <typename T>
__device__ __forceinline__ void st8(T* p, const float v[8]) {
  if constexpr (sizeof(T) == 4) {
    st4<float>(p, v);
    st4<float>(p + 4, v + 4);
  } else {
    *reinterpret_cast<uint4*>(p) = uint4{pk2(v[0], v[1]), pk2(v[2], v[3]), pk2(v[4], v[5]), pk2(v[6], v[7])};
  }
}

// sum of v over the 256 threads of the block (4 waves), returned to every thread
__device__ __forceinline__ float block_sum(float v, float* scratch /* [4] */) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
  __syncthreads();
  return (scratch[0] + scratch[1]) + (scratch[2] + scratch[3]);
}

// ------------------------------------------------------------------ small helpers
// zero up to 16 f32 ranges in one launch (the step's accumulated gradients)
struct ZList {
  int n;
  float* p[17];
  int64_t len[17];
};

// *out += sum over up to 8 f32 ranges of their squares (gradients a stream of the step
// finished writing) or, for ranges added with square = false, of their values (the
// per-workgroup sums of squares a weight-grad GEMM's epilogue left); 16-B lane
// loads, one atomic per block.  The clip's norm so needs no pass over the whole
// gradient buffer after the step's last kernel.
struct SqList {
  int n = 0;
  bool full = false;  // an add past 8 ranges: sq_list refuses the list
  const float* p[8];
  int64_t len[8];
  bool square[8];
  void add(const float* x, int64_t l, bool sq = true) {
    if (n == 8) { full = true; return; }
    p[n] = x; len[n] = l; square[n] = sq; ++n;
  }
};
__global__ __launch_bounds__(256) void sq_list_kernel(SqList q, float* __restrict__ out) {
  __shared__ float part[4];
  float s = 0.f;
  const int64_t gs = (int64_t)gridDim.x * 256, t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (int r = 0; r < q.n; ++r) {
    const float* x = q.p[r];
    const int64_t n = q.len[r];
    if (!q.square[r]) {  // a few hundred GEMM-epilogue partials
      for (int64_t k = t; k < n; k += gs) s += x[k];
      continue;
    }
    const int64_t n4 = ((uintptr_t)x & 15) == 0 ? n / 4 : 0;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    int64_t i = t;
    for (; i + 3 * gs < n4; i += 4 * gs) {
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = x4[i + k * gs];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s = fmaf(v[k].x, v[k].x, s);
        s = fmaf(v[k].y, v[k].y, s);
        s = fmaf(v[k].z, v[k].z, s);
        s = fmaf(v[k].w, v[k].w, s);
      }
    }
    for (; i < n4; i += gs) {
      const float4 v = x4[i];
      s = fmaf(v.x, v.x, s);
      s = fmaf(v.y, v.y, s);
      s = fmaf(v.z, v.z, s);
      s = fmaf(v.w, v.w, s);
    }
    for (int64_t k = 4 * n4 + t; k < n; k += gs) s = fmaf(x[k], x[k], s);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (part[0] + part[1]) + (part[2] + part[3]));
}

static int sq_list(const SqList& q, float* out, hipStream_t st) {
  if (q.full) {
    set_error("nr_latent_train_step: more than 8 grad-norm ranges in one launch");
    return NR_ERR_INVALID;
  }
  if (!out || q.n == 0) return NR_OK;
  int64_t n = 0;
  for (int i = 0; i < q.n; ++i) n += q.len[i];
  const int64_t g = (n / 4 + 1023) / 1024;  // ~4 float4 per thread
  hipLaunchKernelGGL(sq_list_kernel, dim3((unsigned)(g < 1 ? 1 : g < 1024 ? g : 1024)), dim3(256), 0, st, q, out);
  NR_CHECK_LAUNCH("nr_latent_train_step (grad sumsq)");
  return NR_OK;
}
__global__ __launch_bounds__(256) void zero_kernel(ZList z) {
  for (int i = 0; i < z.n; ++i)
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < z.len[i]; k += (int64_t)gridDim.x * 256)
      z.p[i][k] = 0.f;
}

// dst[i] = sum_p src[p * pstride + i] over n contiguous f32 (split-K partials).  Block =
// 64 float4 positions x 4 part groups (group g sums parts g, g + 4, ... in order, the
// four group sums then added in group order: deterministic); the parts' loads spread
// over 4x the threads of one-thread-per-position (the 32-part dlatents sum ran on 64
// blocks at ~0.8 TB/s).  dst may alias src (in place): a block reads all its positions
// before writing them.
__global__ __launch_bounds__(256) void sum_parts_kernel(int64_t n4, int parts, int64_t pstride4,
                                                        const float4* src, float4* dst) {
  __shared__ float4 red[4][64];
  const int pl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + pl;
  float4 v = {0.f, 0.f, 0.f, 0.f};
  if (i < n4)
    for (int p = g; p < parts; p += 4) {
      const float4 w = src[p * pstride4 + i];
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
  red[g][pl] = v;
  __syncthreads();
  if (g == 0 && i < n4) {
    float4 t = red[0][pl];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 w = red[k][pl];
      t.x += w.x; t.y += w.y; t.z += w.z; t.w += w.w;
    }
    dst[i] = t;
  }
}

static int sum_parts(const float* src, int parts, int64_t pstride, float* dst, int64_t n, hipStream_t st) {
  const int64_t n4 = n / 4, g = (n4 + 63) / 64;
  hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)g), dim3(256), 0, st, n4, parts, pstride / 4, (const float4*)src,
                     (float4*)dst);
  NR_CHECK_LAUNCH("nr_latent_train_step (sum_parts)");
  return NR_OK;
}

// ------------------------------------------------------------------ forward rows
// E row of news r: the token LayerNorm (g_mlp_layernorm, eps 1e-12, affine tg / tb)
// of its last token state (TT = f32 / bf16 / f16), the arithmetic of rowops.hip's
// gather_ln_kernel (nr_gather_layernorm): lane's columns 256 j + 4 lane .. +3.  The
// step never stores the [U][1024] E table: the slot gather, the head (pos / neg
// rows) and the LN_q backward recompute the rows they read from the token states.
template <typename TT>
__device__ __forceinline__ void tok_xhat(const TT* __restrict__ row, int lane, float (&v)[4][4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const TT* p = row + j * 256 + lane * 4;
    if constexpr (std::is_same<TT, _Float16>::value) {
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      const h4 h = *reinterpret_cast<const h4*>(p);
      v[j][0] = (float)h[0]; v[j][1] = (float)h[1]; v[j][2] = (float)h[2]; v[j][3] = (float)h[3];
    } else {
      ld4<TT>(p, v[j]);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float d = v[j][t] - mean;
      q = fmaf(d, d, q);
    }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + 1e-12f);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) v[j][t] = (v[j][t] - mean) * rstd;
}
// the E row: xhat tg + tb (the module's affine after tok_xhat's normalisation)
template <typename TT>
__device__ __forceinline__ void tok_ln(const TT* __restrict__ row, int lane, const float* __restrict__ tg,
                                       const float* __restrict__ tb, float (&v)[4][4]) {
  tok_xhat<TT>(row, lane, v);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int e = j * 256 + lane * 4 + t;
      v[j][t] = v[j][t] * tg[e] + tb[e];
    }
}

// Epn rows k < B: E[pos[k]], rows B + k: E[neg[k]] (f32, for the head), and Xpn the
// same rows' token-LN xhat (the head's part of the token LN weight grad).  Wave per row.
template <typename TT>
__global__ __launch_bounds__(256) void pn_rows_kernel(int64_t B, const TT* __restrict__ tok,
                                                      const int32_t* __restrict__ pos, const int32_t* __restrict__ neg,
                                                      const float* __restrict__ tg, const float* __restrict__ tb,
                                                      float* __restrict__ Epn, float* __restrict__ Xpn) {
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= 2 * B) return;  // wave-uniform
  const int64_t r = k < B ? pos[k] : neg[k - B];
  float v[4][4];
  tok_xhat<TT>(tok + r * D, lane, v);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = j * 256 + lane * 4;
    st4<float>(Xpn + k * D + c, v[j]);
    float e[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) e[t] = v[j][t] * tg[c + t] + tb[c + t];
    st4<float>(Epn + k * D + c, e);
  }
}

// Sx = E[idx[row]], X = LN_q(Sx) (eps 1e-5); idx < 0 or row >= nvalid
// (padding): both rows zero.  One wave per row, lane columns 256 j + 4 lane .. +3.
template <typename TA, typename TT>
__global__ __launch_bounds__(256) void gather_ln_kernel(int64_t n, int64_t nvalid, const TT* __restrict__ tok,
                                                        const float* __restrict__ tg, const float* __restrict__ tb,
                                                        const int32_t* __restrict__ idx,
                                                        const float* __restrict__ g, const float* __restrict__ b,
                                                        float eps, TA* __restrict__ Sx, TA* __restrict__ X) {
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += (int64_t)gridDim.x * 4) {
    const int32_t r = row < nvalid ? idx[row] : -1;
    if (r < 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        st4z<TA>(Sx + row * D + j * 256 + lane * 4);
        st4z<TA>(X + row * D + j * 256 + lane * 4);
      }
      continue;
    }
    float v[4][4];
    tok_ln<TT>(tok + (int64_t)r * D, lane, tg, tb, v);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) { const float d = v[j][t] - mean; q = fmaf(d, d, q); }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = j * 256 + lane * 4;
      float o[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = (v[j][t] - mean) * rstd * g[c + t] + b[c + t];
      st4<TA>(Sx + row * D + c, v[j]);
      st4<TA>(X + row * D + c, o);
    }
  }
}

// Per batch row b: zbar_b = mean over its slots of Z = a * gelu(g), (a | g) =
// the two halves of G's 2F columns (GEGLU, latent_attention.py:24-27, exact erf;
// the bf16 step through gelu_erf2x2, |error| <= 3.9e-7), h1bar_b = mean of H1
// (f32), and row_seg[slot] = b.  Z itself is never stored (f32 in registers): its
// only consumer is this mean (m = mean(Z) W2^T + ..., and the backward needs G
// and dZ).  Block = (row b, 256-column chunk: chunks 0..15 of Z, 16..19 of H1);
// the 8 waves stride the segment's rows with 4 rows in flight each, 4 columns
// per lane, fixed-order LDS fold (measured, config-5 step: 512-column chunks and
// 2 rows in flight 66 us; 4 rows, 256 columns 56 us; column chunks as the fast
// grid dimension 48 us; 16 waves 70 us, 8 rows in flight 64 us).  Rows b in
// [B, Bp) of zbar are zero; the last block marks the padding slots -1.
template <typename TA>
__device__ __forceinline__ void geglu4(const float (&a)[4], const float (&g)[4], float (&z)[4]) {
  if constexpr (sizeof(TA) == 4) {
#pragma unroll
    for (int t = 0; t < 4; ++t) z[t] = a[t] * gelu_x(g[t]);
  } else {
    f32x2v g0 = {g[0], g[1]}, g1 = {g[2], g[3]};
    gelu_erf2x2(g0, g1);
    z[0] = a[0] * g0.x; z[1] = a[1] * g0.y; z[2] = a[2] * g1.x; z[3] = a[3] * g1.y;
  }
}

template <typename TA>
__global__ __launch_bounds__(512) void segmean_kernel(int64_t B, int64_t Bp, const int64_t* __restrict__ off,
                                                      int64_t n_rows, const TA* __restrict__ G,
                                                      const TA* __restrict__ H1, TA* __restrict__ zbar,
                                                      float* __restrict__ h1bar, int32_t* __restrict__ row_seg) {
  constexpr int NW = 8, RW = 4, CW = 256, NZ = F / CW;
  __shared__ float part[NW][CW];
  // blockIdx.x = the column chunk: a segment's 20 blocks are dispatched together and
  // read each G row within a short window (DRAM pages / L2 shared), where a
  // chunk-major order touched every G row 32 times, spread over the whole kernel
  const int64_t b = blockIdx.y;
  const int y = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (b >= Bp) {  // the padding slots
    if (y == 0)
      for (int64_t r = off[B] + threadIdx.x; r < n_rows; r += 512) row_seg[r] = -1;
    return;
  }
  const bool zpart = y < NZ;
  const int c0 = (zpart ? y : y - NZ) * CW + lane * 4;
  if (b >= B) {
    if (zpart && wave == 0) st4z<TA>(zbar + b * F + c0);
    return;
  }
  const int64_t r0 = off[b], r1 = off[b + 1];
  if (y == 0)
    for (int64_t r = r0 + threadIdx.x; r < r1; r += 512) row_seg[r] = (int32_t)b;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  // all RW rows' loads issued before any math (rows past the segment re-read its
  // last row and are dropped): a load under a per-row branch is waited on inside it
  for (int64_t r = r0 + wave; r < r1; r += NW * RW) {
    float v[RW][4];
    if (zpart) {
      float a[RW][4], g[RW][4];
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const int64_t ri = min(r + (int64_t)i * NW, r1 - 1);
        ld4<TA>(G + ri * 2 * F + c0, a[i]);
        ld4<TA>(G + ri * 2 * F + F + c0, g[i]);
      }
#pragma unroll
      for (int i = 0; i < RW; ++i) geglu4<TA>(a[i], g[i], v[i]);
    } else {
#pragma unroll
      for (int i = 0; i < RW; ++i) ld4<TA>(H1 + min(r + (int64_t)i * NW, r1 - 1) * D + c0, v[i]);
    }
#pragma unroll
    for (int i = 1; i < RW; ++i)
      if (r + (int64_t)i * NW >= r1)
#pragma unroll
        for (int t = 0; t < 4; ++t) v[i][t] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] += (v[0][t] + v[1][t]) + (v[2][t] + v[3][t]);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) part[wave][lane * 4 + t] = acc[t];
  __syncthreads();
  if (wave != 0) return;
  const float inv = 1.0f / (float)(r1 - r0);  // an empty row gives NaN, as the reference's s / d
  float o[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int c = lane * 4 + t;
    float q[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) q[w] = part[w][c];
#pragma unroll
    for (int h = NW / 2; h > 0; h /= 2)  // pairwise tree, fixed order
#pragma unroll
      for (int w = 0; w < h; ++w) q[w] = q[2 * w] + q[2 * w + 1];
    o[t] = q[0] * inv;
  }
  if (zpart) st4<TA>(zbar + b * F + c0, o);
  else st4<float>(h1bar + b * D + c0, o);
}

// One block per batch row b (256 threads, columns tid + 256 j):
// m = sum_s parts[s][b] + b2 + h1bar[b]; u = m / max(|m|, 1e-12) (F.normalize,
// latent_attention.py:170); F.cosine_similarity(u, E[pos]) / (u, E[neg]) with
// the per-vector 1e-8 clamp and MarginRankingLoss(margin), mean over B
// (trainer.py:1058-1066); backward: du as nr_cosine_margin, dm = (du - u (u .
// du)) / |m| (normalize backward; du / 1e-12 below the clamp).  Writes users = u,
// dmA = dm, dmc = dm / h_b (rows b in [B, Bp): zero; dmc32 = the same in f32: the
// residual of LN_f's backward, where the bf16 dmc -- one rounding shared by all
// h_b slots of the row -- gave the token LN bias grad, whose dominant term is
// sum_b dm_b, a correlated 2^-9 error the bf16 numerics model does not have),
// gb2 += dm, and the pos / neg rows' cosine grads g straight into the token LN's
// parameter grads: gtg += g xhat (Xpn), gtb += g (lane-contiguous atomics: 256 B per
// wave instruction).
template <typename TA>
__global__ __launch_bounds__(256) void head_kernel(int64_t B, int64_t Bp, int nparts, const float* __restrict__ parts,
                                                   const float* __restrict__ b2, const float* __restrict__ h1bar,
                                                   const int64_t* __restrict__ off, const float* __restrict__ Epn,
                                                   float margin,
                                                   float* __restrict__ loss, float* __restrict__ users,
                                                   TA* __restrict__ dmA, TA* __restrict__ dmc,
                                                   float* __restrict__ dmc32, const float* __restrict__ Xpn,
                                                   float* __restrict__ gtg, float* __restrict__ gtb,
                                                   float* __restrict__ gb2) {
  constexpr float EPS = 1e-8f, NEPS = 1e-12f;
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  if (b >= B) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dmA[b * D + j * 256 + tid] = (TA)0.f;
      dmc[b * D + j * 256 + tid] = (TA)0.f;
      dmc32[b * D + j * 256 + tid] = 0.f;
    }
    return;
  }
  float m[4], ep[4], en[4];
  const float* pr = Epn + b * D;         // E[pos[b]]
  const float* nr_ = Epn + (B + b) * D;  // E[neg[b]]
  float mm = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = j * 256 + tid;
    float v = h1bar[b * D + c] + b2[c];
    for (int s = 0; s < nparts; ++s) v += parts[((int64_t)s * Bp + b) * D + c];
    m[j] = v;
    ep[j] = pr[c];
    en[j] = nr_[c];
    mm = fmaf(v, v, mm);
  }
  const float nm = sqrtf(block_sum(mm, red));
  const float den = fmaxf(nm, NEPS);
  float u[4];
  float uu = 0.f, pp = 0.f, nn = 0.f, up = 0.f, un = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    u[j] = m[j] / den;
    uu = fmaf(u[j], u[j], uu);
    pp = fmaf(ep[j], ep[j], pp);
    nn = fmaf(en[j], en[j], nn);
    up = fmaf(u[j], ep[j], up);
    un = fmaf(u[j], en[j], un);
  }
  uu = block_sum(uu, red); pp = block_sum(pp, red); nn = block_sum(nn, red);
  up = block_sum(up, red); un = block_sum(un, red);
  const float nu = sqrtf(uu), np_ = sqrtf(pp), nq = sqrtf(nn);
  const float iu = 1.0f / fmaxf(nu, EPS), ip = 1.0f / fmaxf(np_, EPS), iq = 1.0f / fmaxf(nq, EPS);
  const float sp = up * iu * ip, sn = un * iu * iq;
  const float v = margin - (sp - sn);
  const float act = v >= 0.f ? 1.0f : 0.0f;
  const float gsp = -act / (float)B, gsn = act / (float)B;
  if (tid == 0) atomicAdd(loss, fmaxf(v, 0.f) / (float)B);
  const float cu = nu > EPS ? 1.f : 0.f, cp = np_ > EPS ? 1.f : 0.f, cq = nq > EPS ? 1.f : 0.f;
  const float* xp = Xpn + b * D;         // xhat of E[pos[b]]'s token LN
  const float* xn = Xpn + (B + b) * D;   // and of E[neg[b]]'s
  float g[4];
  float ug = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = j * 256 + tid;
    const float uh = u[j] * iu, ph = ep[j] * ip, qh = en[j] * iq;
    g[j] = gsp * (ph - cu * sp * uh) * iu + gsn * (qh - cu * sn * uh) * iu;
    ug = fmaf(u[j], g[j], ug);
    const float gp = gsp * (uh - cp * sp * ph) * ip, gn = gsn * (uh - cq * sn * qh) * iq;
    atomicAdd(gtg + c, fmaf(gp, xp[c], gn * xn[c]));
    atomicAdd(gtb + c, gp + gn);
  }
  ug = block_sum(ug, red);
  const float icnt = 1.0f / (float)(off[b + 1] - off[b]);
  const bool live = nm > NEPS;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = j * 256 + tid;
    const float dm = (live ? g[j] - u[j] * ug : g[j]) / den;
    atomicAdd(gb2 + c, dm);
    if (users) users[b * D + c] = u[j];
    dmA[b * D + c] = (TA)dm;
    dmc[b * D + c] = (TA)(dm * icnt);
    dmc32[b * D + c] = dm * icnt;
  }
}

// ------------------------------------------------------------------ backward rows
// dG = (dz gelu(g), dz a gelu'(g)) for slot rows, with dz = dZs[row_seg[row]]
// (the per-batch-row dZ of the mean trick, f32, L2-resident), padding slots
// zero; gpart[chunk] = the column sums of dG over the chunk's RB rows (reduced
// over the chunks by nr_col_sum: db1, deterministic).  Block = (RB rows, 512
// a-columns): wave w takes rows RB/4 w .. +RB/4 - 1, all of their G and dZs loads
// issued before any math (4 rows, 128 + 128 B per lane in flight: the two-rows-
// per-iteration loop over 16 rows per thread ran at 3.8 TB/s, latency-bound),
// 8 columns per lane; the waves' column sums fold in LDS in a fixed order.  Row
// chunks, not batch rows: a history length can be ~20x the mean, and one block
// per batch row then waits on the longest.
template <typename TA, int RB>
__global__ __launch_bounds__(256) void geglu_bwd_kernel(int64_t n_rows, const TA* __restrict__ G,
                                                        const float* __restrict__ dZs, const int32_t* __restrict__ row_seg,
                                                        TA* __restrict__ dG, float* __restrict__ gpart) {
  constexpr int RW = RB / 4;  // rows per wave
  __shared__ float red[3][2][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // blockIdx.x = the column chunk (fast): a row chunk's 8 blocks run together
  const int64_t r0 = (int64_t)blockIdx.y * RB + wave * RW;
  const int c = (int)blockIdx.x * 512 + lane * 8;
  int32_t sg_[RW];
  float a[RW][8], g[RW][8], d[RW][8];
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int64_t r = r0 + i;
    sg_[i] = r < n_rows ? row_seg[r] : -2;
  }
  // every row's loads issued unconditionally (clamped row / segment 0 for the
  // padding): a load under a per-row branch is waited on inside that branch
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int64_t r = min(r0 + i, n_rows - 1);
    ld8<TA>(G + r * 2 * F + c, a[i]);
    ld8<TA>(G + r * 2 * F + F + c, g[i]);
    ld8<float>(dZs + (int64_t)max(sg_[i], 0) * F + c, d[i]);
  }
  float sa[8], sg[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { sa[k] = 0.f; sg[k] = 0.f; }
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int64_t r = r0 + i;
    if (sg_[i] >= 0) {
      float da[8], dg[8];
#pragma unroll
      for (int k = 0; k < 8; k += 2) {
        float cdf[2], pdf[2];
        if constexpr (sizeof(TA) == 4) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            cdf[j] = 0.5f * (1.0f + erff(g[i][k + j] * 0.70710678118654752440f));
            pdf[j] = 0.39894228040143267794f * expf(-0.5f * g[i][k + j] * g[i][k + j]);  // exact f32, as the forward
          }
        } else {
          f32x2v h, e;
          erfc_half2((f32x2v){g[i][k], g[i][k + 1]}, h, e);
          cdf[0] = g[i][k] >= 0.f ? 1.0f - h.x : h.x;
          cdf[1] = g[i][k + 1] >= 0.f ? 1.0f - h.y : h.y;
          pdf[0] = 0.39894228040143267794f * e.x;
          pdf[1] = 0.39894228040143267794f * e.y;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float gk = g[i][k + j], dk = d[i][k + j];
          da[k + j] = dk * gk * cdf[j];
          dg[k + j] = dk * a[i][k + j] * (cdf[j] + gk * pdf[j]);
          sa[k + j] += da[k + j];
          sg[k + j] += dg[k + j];
        }
      }
      st8<TA>(dG + r * 2 * F + c, da);
      st8<TA>(dG + r * 2 * F + F + c, dg);
    } else if (sg_[i] == -1) {
      const float zero[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      st8<TA>(dG + r * 2 * F + c, zero);
      st8<TA>(dG + r * 2 * F + F + c, zero);
    }
  }
  if (wave > 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { red[wave - 1][0][lane * 8 + k] = sa[k]; red[wave - 1][1][lane * 8 + k] = sg[k]; }
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int j = lane * 8 + k;
    sa[k] = (sa[k] + red[0][0][j]) + (red[1][0][j] + red[2][0][j]);
    sg[k] = (sg[k] + red[0][1][j]) + (red[1][1][j] + red[2][1][j]);
  }
  st8<float>(gpart + (int64_t)blockIdx.y * 2 * F + c, sa);
  st8<float>(gpart + (int64_t)blockIdx.y * 2 * F + F + c, sg);
}

// LayerNorm input gradient (stats recomputed from x with the forward's
// arithmetic) plus a residual gradient, and the LN parameter grads:
//   dx = rstd (dxh - mean(dxh) - xhat mean(dxh xhat)) + res,  dxh = dy gamma
//   dgamma += dy xhat, dbeta += dy (per-lane registers, one atomic per column per block)
// MODE 0 (LN_f of H1): res = dmc32[row_seg[row]] (f32: the broadcast dH of the mean),
//   dx -> out rows (TA); padding slots (row_seg < 0) -> zero rows.
// MODE 1 (LN_q of S):  x = the f32 row E[idx[row]] the forward normalised (tok_ln of
//   the token row tokv[idx[row]], not the bf16-stored S: the statistics of the rounded row moved the token LN
//   bias grad ~10x past the bf16 numerics model's drift, test_train_bf16_drift),
//   res = dH1 row (TA); dx = the slot's gradient of its E row, which only the token
//   LN's parameters consume: tdg += dx xhat_tok, tdb += dx (per-lane registers, one
//   atomic per column per block, as dgamma / dbeta), in place of a [U][1024] dE
//   scatter (8.5 M f32 atomics at the benchmark batch) and a pass over it; idx < 0
//   skipped.
template <typename TA, int MODE, typename TT = float>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int64_t n, int64_t nvalid, const TA* __restrict__ x,
                                                     const void* __restrict__ tokv, const float* __restrict__ gamma,
                                                     float eps,
                                                     const TA* __restrict__ dy, const void* __restrict__ res_,
                                                     const int32_t* __restrict__ sel, TA* __restrict__ out,
                                                     float* __restrict__ tdg, float* __restrict__ tdb,
                                                     float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                     const float* __restrict__ tg, const float* __restrict__ tb) {
  __shared__ float sg[4][D], sb[4][D];
  constexpr int NT = MODE == 1 ? 4 : 1;  // token-LN grad accumulators (MODE 1)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float ag[4][4], ab[4][4], gm[4][4], tga[NT][4], tba[NT][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ld4<float>(gamma + j * 256 + lane * 4, gm[j]);
#pragma unroll
    for (int t = 0; t < 4; ++t) { ag[j][t] = 0.f; ab[j][t] = 0.f; }
  }
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) { tga[j][t] = 0.f; tba[j][t] = 0.f; }
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < n; row += (int64_t)gridDim.x * 4) {
    const int32_t s = row < nvalid ? sel[row] : -1;
    if (s < 0) {
      if constexpr (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) st4z<TA>(out + row * D + j * 256 + lane * 4);
      }
      continue;
    }
    // x, dy and the residual row issued together (one memory round trip per row;
    // dy and res behind the statistics' reductions made the kernel latency-bound)
    float v[4][4], g[4][4], dyv[4][4], rv[4][4], xt[NT][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = j * 256 + lane * 4;
      if constexpr (MODE == 0) ld4<TA>(x + row * D + c, v[j]);
      ld4<TA>(dy + row * D + c, dyv[j]);
      if constexpr (MODE == 0) ld4<float>(static_cast<const float*>(res_) + (int64_t)s * D + c, rv[j]);
      else ld4<TA>(static_cast<const TA*>(res_) + row * D + c, rv[j]);
    }
    if constexpr (MODE == 1) {
      tok_xhat<TT>(static_cast<const TT*>(tokv) + (int64_t)s * D, lane, xt);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int e = j * 256 + lane * 4 + t;
          v[j][t] = xt[j][t] * tg[e] + tb[e];
        }
    }
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) sum += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
    const float mean = wave_sum(sum) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) { const float d = v[j][t] - mean; q = fmaf(d, d, q); }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* d4 = dyv[j];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v[j][t] = (v[j][t] - mean) * rstd;  // xhat
        ag[j][t] = fmaf(d4[t], v[j][t], ag[j][t]);
        ab[j][t] += d4[t];
        g[j][t] = d4[t] * gm[j][t];  // dxhat
        s1 += g[j][t];
        s2 = fmaf(g[j][t], v[j][t], s2);
      }
    }
    const float m1 = wave_sum(s1) / (float)D, m2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = j * 256 + lane * 4;
      float o[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = rstd * (g[j][t] - m1 - v[j][t] * m2) + rv[j][t];
      if constexpr (MODE == 0) {
        st4<TA>(out + row * D + c, o);
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          tga[j][t] = fmaf(o[t], xt[j][t], tga[j][t]);
          tba[j][t] += o[t];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sg[wave][j * 256 + lane * 4 + t] = ag[j][t];
      sb[wave][j * 256 + lane * 4 + t] = ab[j][t];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    atomicAdd(dgamma + c, (sg[0][c] + sg[1][c]) + (sg[2][c] + sg[3][c]));
    atomicAdd(dbeta + c, (sb[0][c] + sb[1][c]) + (sb[2][c] + sb[3][c]));
  }
  if constexpr (MODE == 1) {  // the token LN's grads, the same way
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        sg[wave][j * 256 + lane * 4 + t] = tga[j][t];
        sb[wave][j * 256 + lane * 4 + t] = tba[j][t];
      }
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256) {
      atomicAdd(tdg + c, (sg[0][c] + sg[1][c]) + (sg[2][c] + sg[3][c]));
      atomicAdd(tdb + c, (sb[0][c] + sb[1][c]) + (sb[2][c] + sb[3][c]));
    }
  }
}

// dS = P (dP - sum_group P dP) over the 8 groups of 64 columns (one head's
// latents, SDPA's softmax backward).  One wave per (row, group).
template <typename TA>
__global__ __launch_bounds__(256) void softmax64_bwd_kernel(int64_t rows, const TA* __restrict__ P,
                                                            const TA* __restrict__ dP, TA* __restrict__ dS) {
  const int lane = threadIdx.x & 63;
  const int64_t ng = rows * HEADS;
  for (int64_t gi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); gi < ng; gi += (int64_t)gridDim.x * 4) {
    const int64_t i = gi * 64 + lane;  // rows x 512 = groups x 64
    const float p = (float)P[i], d = (float)dP[i];
    const float dot = wave_sum(p * d);
    dS[i] = (TA)(p * (d - dot));
  }
}

// Backward of the latents' LayerNorm (norm_context, 64 rows) with dy = the sum
// of `ns` split-K partials [ns][64][1024]: one wave per row (16 blocks),
// dlatents written, dgamma / dbeta accumulated (one atomic per column per block).
__global__ __launch_bounds__(256) void lnc_bwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                      float eps, int ns, const float* __restrict__ parts,
                                                      float* __restrict__ dx, float* __restrict__ dgamma,
                                                      float* __restrict__ dbeta) {
  __shared__ float sg[4][D], sb[4][D];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = (int)blockIdx.x * 4 + wave;  // 16 blocks x 4 waves = the 64 latents
  float v[4][4], g[4][4], dy[4][4];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = j * 256 + lane * 4;
    ld4<float>(x + row * D + c, v[j]);
    sum += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
#pragma unroll
    for (int t = 0; t < 4; ++t) dy[j][t] = 0.f;
    for (int s = 0; s < ns; ++s) {
      float p4[4];
      ld4<float>(parts + ((int64_t)s * NL + row) * D + c, p4);
#pragma unroll
      for (int t = 0; t < 4; ++t) dy[j][t] += p4[t];
    }
  }
  const float mean = wave_sum(sum) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) { const float d = v[j][t] - mean; q = fmaf(d, d, q); }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float gm[4];
    ld4<float>(gamma + j * 256 + lane * 4, gm);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      v[j][t] = (v[j][t] - mean) * rstd;
      sg[wave][j * 256 + lane * 4 + t] = dy[j][t] * v[j][t];
      sb[wave][j * 256 + lane * 4 + t] = dy[j][t];
      g[j][t] = dy[j][t] * gm[t];
      s1 += g[j][t];
      s2 = fmaf(g[j][t], v[j][t], s2);
    }
  }
  const float m1 = wave_sum(s1) / (float)D, m2 = wave_sum(s2) / (float)D;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = rstd * (g[j][t] - m1 - v[j][t] * m2);
    st4<float>(dx + row * D + j * 256 + lane * 4, o);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    atomicAdd(dgamma + c, (sg[0][c] + sg[1][c]) + (sg[2][c] + sg[3][c]));
    atomicAdd(dbeta + c, (sb[0][c] + sb[1][c]) + (sb[2][c] + sb[3][c]));
  }
}

// ------------------------------------------------------------------ batched transposes
// Up to kTMax matrices per launch (the step's weight transposes, the weight-grad
// operands, the fold's operands): dst = src^T (transpose = 1) or dst = src
// (a dtype conversion), 64 x 64 tiles.  A source may be `parts` f32 split-K
// planes (pstride elements apart) that are summed on the way.  rows_pad >= rows:
// a transposed dst gets zero columns [rows, rows_pad) (the zero K tail of a
// split-K weight-grad GEMM).
constexpr int kTMax = 8;
struct TBatch {
  int n;
  int tile_end[kTMax], tiles_x[kTMax], transpose[kTMax], parts[kTMax];
  const void* src[kTMax];
  void* dst[kTMax];
  int64_t rows[kTMax], rows_pad[kTMax], cols[kTMax], lds[kTMax], ldd[kTMax], pstride[kTMax];
};

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void transpose_batched_kernel(TBatch tb) {
  __shared__ float tile[64][65];
  const int t = (int)blockIdx.x;
  int p = 0;
  while (p + 1 < tb.n && t >= tb.tile_end[p]) ++p;
  const int local = t - (p ? tb.tile_end[p - 1] : 0);
  const int64_t r0 = (int64_t)(local / tb.tiles_x[p]) * 64, c0 = (int64_t)(local % tb.tiles_x[p]) * 64;
  const TI* src = (const TI*)tb.src[p];
  TO* dst = (TO*)tb.dst[p];
  const int64_t rows = tb.rows[p], rpad = tb.rows_pad[p], cols = tb.cols[p], lds = tb.lds[p], ldd = tb.ldd[p];
  const int np = tb.parts[p];
  const int64_t ps = tb.pstride[p];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  auto val = [&](int64_t r, int64_t c) {
    float v = (float)src[r * lds + c];
    for (int q = 1; q < np; ++q) v += (float)src[q * ps + r * lds + c];
    return v;
  };
  if (!tb.transpose[p]) {
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
      const int64_t r = r0 + ty + 4 * k, c = c0 + tx;
      if (r < rows && c < cols) dst[r * ldd + c] = (TO)val(r, c);
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int rr = ty + 4 * k;
    const int64_t r = r0 + rr, c = c0 + tx;
    tile[rr][tx] = (r < rows && c < cols) ? val(r, c) : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int cc = ty + 4 * k;
    const int64_t c = c0 + cc, r = r0 + tx;
    if (c < cols && r < rpad) dst[c * ldd + r] = (TO)tile[tx][cc];
  }
}

// 16-bit -> 16-bit transposes with 16-B global accesses (train.hip's
// transpose16_kernel, batched): rows_pad / cols / strides multiples of 8.
__global__ __launch_bounds__(256) void transpose16_batched_kernel(TBatch tb) {
  constexpr int P = 66;
  __shared__ uint16_t tile[64 * P];
  const int t = (int)blockIdx.x;
  int p = 0;
  while (p + 1 < tb.n && t >= tb.tile_end[p]) ++p;
  const int local = t - (p ? tb.tile_end[p - 1] : 0);
  const int64_t r0 = (int64_t)(local / tb.tiles_x[p]) * 64, c0 = (int64_t)(local % tb.tiles_x[p]) * 64;
  const uint16_t* src = (const uint16_t*)tb.src[p];
  uint16_t* dst = (uint16_t*)tb.dst[p];
  const int64_t rows = tb.rows[p], rpad = tb.rows_pad[p], cols = tb.cols[p], lds = tb.lds[p], ldd = tb.ldd[p];
  const int th = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int rr = (th >> 3) + 32 * k, ch = th & 7;
    const int64_t r = r0 + rr, c = c0 + 8 * ch;
    uint4 u = make_uint4(0, 0, 0, 0);
    if (r < rows && c < cols) u = *reinterpret_cast<const uint4*>(src + r * lds + c);
    uint32_t* d = reinterpret_cast<uint32_t*>(tile + rr * P + 8 * ch);
    d[0] = u.x; d[1] = u.y; d[2] = u.z; d[3] = u.w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int oc = (th >> 3) + 32 * k, rc = th & 7;
    const int64_t c = c0 + oc, r = r0 + 8 * rc;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)tile[(8 * rc + 2 * j) * P + oc] | ((uint32_t)tile[(8 * rc + 2 * j + 1) * P + oc] << 16);
    if (c < cols && r < rpad) *reinterpret_cast<uint4*>(dst + c * ldd + r) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

struct TList {
  TBatch b{};
  int tiles = 0;
  bool all16 = true;
  void add(const void* src, int64_t lds, void* dst, int64_t ldd, int64_t rows, int64_t cols, bool tr,
           int64_t rows_pad = 0, int parts = 1, int64_t pstride = 0) {
    const int i = b.n++;
    if (rows_pad < rows) rows_pad = rows;
    b.src[i] = src; b.dst[i] = dst; b.rows[i] = rows; b.rows_pad[i] = rows_pad; b.cols[i] = cols;
    b.lds[i] = lds; b.ldd[i] = ldd; b.parts[i] = parts; b.pstride[i] = pstride;
    b.transpose[i] = tr ? 1 : 0;
    b.tiles_x[i] = (int)((cols + 63) / 64);
    tiles += (int)(((rows_pad + 63) / 64) * b.tiles_x[i]);
    b.tile_end[i] = tiles;
    all16 = all16 && tr && parts == 1 && rows_pad % 8 == 0 && cols % 8 == 0 && lds % 8 == 0 && ldd % 8 == 0;
  }
};

// TI -> TO batched transposes / conversions; 16-bit to 16-bit transposes on the 16-B kernel
template <typename TI, typename TO>
int launch_tlist(const TList& l, hipStream_t s) {
  if (l.b.n == 0) return NR_OK;
  if (sizeof(TI) == 2 && sizeof(TO) == 2 && l.all16)
    hipLaunchKernelGGL(transpose16_batched_kernel, dim3((unsigned)l.tiles), dim3(256), 0, s, l.b);
  else
    hipLaunchKernelGGL((transpose_batched_kernel<TI, TO>), dim3((unsigned)l.tiles), dim3(256), 0, s, l.b);
  NR_CHECK_LAUNCH("nr_latent_train_step (transposes)");
  return NR_OK;
}

// f32 split-K partials -> their sum in TO twice, as is (plain) and transposed:
// the fold's operands (KV / KV^T, gA / gA^T, gBt / gBt^T, dKV / dKV^T).  One
// 32-row x 64-column tile per block (64-row tiles: half the blocks, ~12 us/step
// slower in an interleaved A/B, profiles/round5/train/ab_r8a), up to kSCMax
// matrices per launch: each partial is read once with 16-B loads, all `parts`
// loads of a row issued together, the sum in slice order, the plain tile stored
// from registers and the transposed one through LDS.  The generic TBatch path read
// every partial twice (once per output) with 4-B loads: 34-38 us for the gA / gBt set.
constexpr int kSCMax = 2;
struct SCBatch {
  int n;
  int tile_end[kSCMax], tiles_x[kSCMax], parts[kSCMax];
  const float* src[kSCMax];
  void* plain[kSCMax];
  void* trans[kSCMax];
  int64_t cols[kSCMax], lds[kSCMax], ldp[kSCMax], ldt[kSCMax], pstride[kSCMax];
};

template <typename TO>
__global__ __launch_bounds__(256) void sumconv_kernel(SCBatch sb) {
  __shared__ float tile[32][65];
  const int t = (int)blockIdx.x;
  int p = 0;
  while (p + 1 < sb.n && t >= sb.tile_end[p]) ++p;
  const int local = t - (p ? sb.tile_end[p - 1] : 0);
  const int64_t r0 = (int64_t)(local / sb.tiles_x[p]) * 32, c0 = (int64_t)(local % sb.tiles_x[p]) * 64;
  const float* src = sb.src[p];
  const int np = sb.parts[p];
  const int64_t lds = sb.lds[p], ps = sb.pstride[p];
  const int th = threadIdx.x, rg = th >> 4, c4 = (th & 15) * 4;
  TO* plain = (TO*)sb.plain[p];
  const int64_t ldp = sb.ldp[p];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int rr = rg + 16 * k;
    const float* s = src + (r0 + rr) * lds + c0 + c4;
    float4 v = *reinterpret_cast<const float4*>(s);
#pragma unroll 8
    for (int q = 1; q < np; ++q) {
      const float4 w = *reinterpret_cast<const float4*>(s + q * ps);
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
    const float o[4] = {v.x, v.y, v.z, v.w};
    st4<TO>(plain + (r0 + rr) * ldp + c0 + c4, o);
    tile[rr][c4] = v.x; tile[rr][c4 + 1] = v.y; tile[rr][c4 + 2] = v.z; tile[rr][c4 + 3] = v.w;
  }
  __syncthreads();
  TO* trans = (TO*)sb.trans[p];
  const int64_t ldt = sb.ldt[p];
  {
    const int cc = th >> 2, rc = (th & 3) * 8;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = tile[rc + j][cc];
    st8<TO>(trans + (c0 + cc) * ldt + r0 + rc, o);
  }
}

struct SCList {
  SCBatch b{};
  int tiles = 0;
  // src [rows, cols] (ld lds, `parts` slices pstride apart) -> plain [rows, cols] (ld ldp)
  // and trans [cols, rows] (ld ldt); rows, cols multiples of 64
  int add(const float* src, int64_t lds, int parts, int64_t pstride, int64_t rows, int64_t cols, void* plain,
          int64_t ldp, void* trans, int64_t ldt) {
    if (b.n >= kSCMax || rows % 64 || cols % 64 || lds % 4 || pstride % 4 || ldp % 8 || ldt % 8) {
      set_error("nr_latent_train_step: sumconv operand %d: rows %lld / cols %lld not multiples of 64", b.n,
                (long long)rows, (long long)cols);
      return NR_ERR_INVALID;
    }
    const int i = b.n++;
    b.src[i] = src; b.plain[i] = plain; b.trans[i] = trans; b.parts[i] = parts; b.pstride[i] = pstride;
    b.cols[i] = cols; b.lds[i] = lds; b.ldp[i] = ldp; b.ldt[i] = ldt;
    b.tiles_x[i] = (int)(cols / 64);
    tiles += (int)(rows / 32 * (cols / 64));
    b.tile_end[i] = tiles;
    return NR_OK;
  }
};

template <typename TO>
int launch_sumconv(const SCList& l, hipStream_t s) {
  if (l.b.n == 0) return NR_OK;
  hipLaunchKernelGGL((sumconv_kernel<TO>), dim3((unsigned)l.tiles), dim3(256), 0, s, l.b);
  NR_CHECK_LAUNCH("nr_latent_train_step (sumconv)");
  return NR_OK;
}

static int64_t pad64(int64_t n) { return n < 64 ? 64 : (n + 63) / 64 * 64; }
static int64_t al(int64_t b) { return (b + 255) / 256 * 256; }

constexpr int kKVParts = 4;    // split-K slices of KV = latn Wkv^T (K = 1024 -> 256)
constexpr int kHParts = 16;    // split-K slices of the m GEMM (K = 4096 -> 256)
constexpr int kZParts = 4;     // split-K slices of dZ = dmc W2 (K = 1024 -> 256)
constexpr int kGRows = 16;     // slot rows per GEGLU-backward block
constexpr int kWParts = 8;     // split-K slices of dA / dBt (K = Hp -> Hpp / 8)
constexpr int kLatParts = 32;  // split-K slices of dlatents' GEMM (K = 8192 -> 256)
// per-workgroup sum-of-squares slots of the weight-grad GEMMs (the clip's norm):
// dW1 / dW2 (192 workgroups), the fold group (160), dWkv + dlatents (256)
constexpr int kSqW12 = 0, kSqFold = 320, kSqKv = 512, kSqSlots = 832;

// Workspace layout (byte offsets), shared by the size query and the step.
struct Layout {
  int64_t Hp, Hpp, kw, Bp, es;
  int64_t E, Xpn, Sx, X, P, H1, Y, G, zbar, h1bar, row_seg, hparts, hsum, dmA, dmc, dmc32, dZ, dZs, gpart, dG, dY, dH1,
      dP, dS, dX;
  int64_t dGT, YT, dH1T, PT, dST, XT, dmT, zbarT;
  int64_t WqT, W1T, W2T, WoT, WkvT, latn, latnT, KVp, KV, KVT, A, AT, BtT, Bt;
  int64_t gA, gBt, gA16, gAT16, gBt16, gBtT16, dKV, dKV16, dKVT16, dlat, sqp;
  int64_t total;
};

static Layout layout(int dtype, int64_t B, int64_t U, int64_t Hs) {
  Layout L{};
  L.Hp = pad64(Hs);
  // dA / dBt run as kWParts K-slices of kw rows: Hpp = kWParts kw >= Hp (zero columns past Hp)
  L.kw = (L.Hp / 64 + kWParts - 1) / kWParts * 64;
  L.Hpp = L.kw * kWParts;
  L.Bp = pad64(B);
  L.es = dtype == NR_F32 ? 4 : 2;
  const int64_t Hp = L.Hp, Hpp = L.Hpp, Bp = L.Bp, es = L.es;
  int64_t o = 0;
  auto take = [&](int64_t bytes) { const int64_t r = o; o += al(bytes); return r; };
  L.E = take(2 * Bp * D * 4);  // Epn: E[pos] rows then E[neg] rows (no [U][D] E table)
  L.Xpn = take(2 * Bp * D * 4);  // the same rows' token-LN xhat
  // X, P, dH1, dS hold Hpp rows: the dA / dBt K-slices read them directly (bf16: TN
  // weight-grad GEMMs), rows [Hp, Hpp) zeroed by the step
  L.Sx = take(Hp * D * es); L.X = take(Hpp * D * es); L.P = take(Hpp * S * es); L.H1 = take(Hp * D * es);
  L.Y = take(Hp * D * es); L.G = take(Hp * 2 * F * es);
  L.zbar = take(Bp * F * es); L.h1bar = take(Bp * D * 4); L.row_seg = take(Hp * 4);
  L.hparts = take((int64_t)kHParts * Bp * D * 4); L.hsum = take(Bp * D * 4);
  L.dmA = take(Bp * D * es); L.dmc = take(Bp * D * es); L.dmc32 = take(Bp * D * 4); L.dZ = take((int64_t)kZParts * Bp * F * 4);
  L.dZs = take(Bp * F * 4);
  L.gpart = take((Hp + kGRows - 1) / kGRows * 2 * F * 4);
  L.dG = take(Hp * 2 * F * es); L.dY = take(Hp * D * es); L.dH1 = take(Hpp * D * es);
  L.dP = take(Hp * S * es); L.dS = take(Hpp * S * es); L.dX = take(Hp * D * es);
  L.dGT = take(2 * F * Hp * es); L.YT = take(D * Hp * es); L.dH1T = take(D * Hpp * es); L.PT = take(S * Hpp * es);
  L.dST = take(S * Hpp * es); L.XT = take(D * Hpp * es); L.dmT = take(D * Bp * es); L.zbarT = take(F * Bp * es);
  L.WqT = take(D * F * es); L.W1T = take(D * 2 * F * es); L.W2T = take(F * D * es); L.WoT = take(F * D * es);
  L.WkvT = take(D * 2 * F * es);
  L.latn = take(NL * D * es); L.latnT = take(D * NL * es); L.KVp = take((int64_t)kKVParts * NL * 2 * F * 4);
  L.KV = take(NL * 2 * F * es); L.KVT = take(2 * F * NL * es);
  L.A = take(S * D * es); L.AT = take(D * S * es); L.BtT = take(S * D * es); L.Bt = take(D * S * es);
  L.gA = take((int64_t)kWParts * S * D * 4); L.gBt = take((int64_t)kWParts * D * S * 4);
  L.gA16 = take(S * D * es); L.gAT16 = take(D * S * es); L.gBt16 = take(D * S * es); L.gBtT16 = take(S * D * es);
  L.dKV = take(NL * 2 * F * 4); L.dKV16 = take(NL * 2 * F * es); L.dKVT16 = take(2 * F * NL * es);
  L.dlat = take((int64_t)kLatParts * NL * D * 4);
  L.sqp = take(kSqSlots * 4);
  L.total = o;
  return L;
}

static int grid_rows(int64_t rows, int cap = 1024) {
  const int64_t g = (rows + 3) / 4;
  return (int)(g < cap ? (g > 0 ? g : 1) : cap);
}

template <typename TA>
int step(const nr_latent_train_args& a, char* ws, hipStream_t st) {
  const int dt = a.dtype;
  const Layout L = layout(dt, a.B, a.U, a.Hs);
  const int64_t B = a.B, Hp = L.Hp, Hpp = L.Hpp, Bp = L.Bp;
  auto P_ = [&](int64_t off) { return (void*)(ws + off); };
  float* Epn = (float*)P_(L.E);
  float* Xpn = (float*)P_(L.Xpn);
  TA *Sx = (TA*)P_(L.Sx), *X = (TA*)P_(L.X), *Pm = (TA*)P_(L.P), *H1 = (TA*)P_(L.H1), *Y = (TA*)P_(L.Y);
  TA *G = (TA*)P_(L.G), *zbar = (TA*)P_(L.zbar);
  float* h1bar = (float*)P_(L.h1bar);
  int32_t* row_seg = (int32_t*)P_(L.row_seg);
  float* hparts = (float*)P_(L.hparts);
  float* hsum = (float*)P_(L.hsum);
  float* dZs = (float*)P_(L.dZs);
  TA *dmA = (TA*)P_(L.dmA), *dmc = (TA*)P_(L.dmc);
  float* dmc32 = (float*)P_(L.dmc32);
  float* dZ = (float*)P_(L.dZ);
  float* gpart = (float*)P_(L.gpart);
  TA *dG = (TA*)P_(L.dG), *dY = (TA*)P_(L.dY), *dH1 = (TA*)P_(L.dH1), *dP = (TA*)P_(L.dP), *dS = (TA*)P_(L.dS);
  TA* dX = (TA*)P_(L.dX);
  TA *dGT = (TA*)P_(L.dGT), *YT = (TA*)P_(L.YT), *dH1T = (TA*)P_(L.dH1T), *PT = (TA*)P_(L.PT), *dST = (TA*)P_(L.dST);
  TA *XT = (TA*)P_(L.XT), *dmT = (TA*)P_(L.dmT), *zbarT = (TA*)P_(L.zbarT);
  TA *WqT = (TA*)P_(L.WqT), *W1T = (TA*)P_(L.W1T), *W2T = (TA*)P_(L.W2T), *WoT = (TA*)P_(L.WoT),
     *WkvT = (TA*)P_(L.WkvT);
  TA *latn = (TA*)P_(L.latn), *latnT = (TA*)P_(L.latnT), *KV = (TA*)P_(L.KV), *KVT = (TA*)P_(L.KVT);
  float* KVp = (float*)P_(L.KVp);
  TA *Am = (TA*)P_(L.A), *AT = (TA*)P_(L.AT), *BtT = (TA*)P_(L.BtT), *Bt = (TA*)P_(L.Bt);
  float *gA = (float*)P_(L.gA), *gBt = (float*)P_(L.gBt);
  TA *gA16 = (TA*)P_(L.gA16), *gAT16 = (TA*)P_(L.gAT16), *gBt16 = (TA*)P_(L.gBt16), *gBtT16 = (TA*)P_(L.gBtT16);
  float* dKV = (float*)P_(L.dKV);
  TA *dKV16 = (TA*)P_(L.dKV16), *dKVT16 = (TA*)P_(L.dKVT16);
  float* dlat = (float*)P_(L.dlat);
  float* sqp = a.sumsq ? (float*)P_(L.sqp) : nullptr;  // GEMM-epilogue sum-of-squares slots
  int n_sq12 = 0, n_sqf = 0, n_sqkv = 0;
  const TA *Wq = (const TA*)a.Wq, *Wkv = (const TA*)a.Wkv, *Wo = (const TA*)a.Wo, *W1 = (const TA*)a.W1,
           *W2 = (const TA*)a.W2;
  const float scale = 1.0f / sqrtf((float)DH);  // SDPA default scale (latent_attention.py:72)
  TrainSide side;
  int rc;
  if ((rc = train_side_streams(st, "nr_latent_train_step", side))) return rc;
#define NR_LT_CHECK(name) NR_CHECK_LAUNCH("nr_latent_train_step (" name ")")

  // ---- fork 0: the fold (weights only) runs on the side stream beside Wq^T, the
  // token LN, the history gather and the data-grad weight transposes on this one
  // (interleaved A/B: Wq^T here 1.045-1.055 vs on the fold stream 1.053-1.061 ms/step,
  // profiles/round5/train/ab_r8c); the P GEMM joins them.  The side stream first waits for everything before the step on
  // this one (the previous step's AdamW rewrote the weights).
  if (hipEventRecord(side.fork, st) != hipSuccess || hipStreamWaitEvent(side.s, side.fork, 0) != hipSuccess) {
    set_error("nr_latent_train_step: fork 0 failed");
    return NR_ERR_HIP;
  }
  // Wq^T (the A fold's operand) first on this stream, event wt: the fold stream runs
  // LN_c and the KV GEMM meanwhile and waits for it just before the A / Bt GEMMs
  {
    TList t;
    t.add(Wq, D, WqT, F, F, D, true);  // [4096, 1024] -> [1024, 4096]
    if ((rc = launch_tlist<TA, TA>(t, st))) return rc;
    if (hipEventRecord(side.wt, st) != hipSuccess) {
      set_error("nr_latent_train_step: Wq transpose record failed");
      return NR_ERR_HIP;
    }
  }
  // the data-grad GEMMs' W operands (first needed by the dZ GEMM), on this stream
  // before the gathers: beside LN_c and the KV GEMM rather than the A / Bt GEMMs, and
  // not beside the P GEMM (interleaved A/B: 1.090-1.095 vs after the gathers
  // 1.097-1.102 ms/step, profiles/round5/train/ab_r8f)
  {
    TList t;
    t.add(W1, D, W1T, 2 * F, 2 * F, D, true);  // [8192, 1024] -> [1024, 8192]
    t.add(W2, F, W2T, D, D, F, true);          // [1024, 4096] -> [4096, 1024]
    t.add(Wo, F, WoT, D, D, F, true);          // [1024, 4096] -> [4096, 1024]
    t.add(Wkv, D, WkvT, 2 * F, 2 * F, D, true);
    if ((rc = launch_tlist<TA, TA>(t, st))) return rc;
  }
  // ---- accumulators: the step zeroes every gradient it accumulates (the GEMM-written
  // ones are overwritten whole) and the loss
  {
    ZList z{};
    float* zp[] = {a.g_tok_g, a.g_tok_b, a.g_nq_g, a.g_nq_b, a.g_nc_g, a.g_nc_b, a.g_nf_g, a.g_nf_b, a.g_b2, a.g_b1, a.loss};
    const int64_t zn[] = {D, D, D, D, D, D, D, D, D, 2 * F, 1};
    for (int i = 0; i < 11; ++i) { z.p[i] = zp[i]; z.len[i] = zn[i]; }
    // rows [Hp, Hpp) of the dA / dBt operands (read as the K-slices' zero tail)
    const int64_t tail = (Hpp - Hp) * L.es / 4;  // in f32 words (Hpp - Hp is a multiple of 64 rows)
    z.p[11] = (float*)(X + Hp * D); z.len[11] = tail * D;
    z.p[12] = (float*)(Pm + Hp * S); z.len[12] = tail * S;
    z.p[13] = (float*)(dH1 + Hp * D); z.len[13] = tail * D;
    z.p[14] = (float*)(dS + Hp * S); z.len[14] = tail * S;
    z.n = 15;
    if (a.sumsq) { z.p[15] = a.sumsq; z.len[15] = 1; z.n = 16; }
    hipLaunchKernelGGL(zero_kernel, dim3(1024), dim3(256), 0, st, z);
    NR_LT_CHECK("zero");
  }
  // (one box, interleaved, ms/step: all of this serial on one stream 1.195-1.215, every
  // weight transpose before the fold on the side stream 1.20, this layout 1.185 --
  // profiles/round4/train/step_tuning/r4ab1)
  hipStream_t fs = side.s;
  // fold: latn = LN_c(latents); KV = latn Wkv^T (split-K); A_h = s K_h Wq_h; BtT_h = V_h Wo_h^T
  if ((rc = layernorm_dispatch(NR_F32, dt, NL, D, a.latents, D, a.nc_g, a.nc_b, 1e-5f, latn, D, fs))) return rc;
  {
    const int64_t ks = D / kKVParts;
    GemmProblem p = {NL, 2 * F, ks, latn, D, ks, Wkv, D, ks, KVp, 2 * F, (int64_t)NL * 2 * F, kKVParts, 1.0f};
    if ((rc = gemm_group_dispatch(dt, NR_F32, &p, 1, fs))) return rc;
    SCList t;
    if ((rc = t.add(KVp, 2 * F, kKVParts, (int64_t)NL * 2 * F, NL, 2 * F, KV, 2 * F, KVT, NL))) return rc;
    if ((rc = launch_sumconv<TA>(t, fs))) return rc;
  }
  if (hipStreamWaitEvent(fs, side.wt, 0) != hipSuccess) {
    set_error("nr_latent_train_step: Wq transpose wait failed");
    return NR_ERR_HIP;
  }
  {
    GemmProblem p[2] = {
        {NL, D, DH, KV, 2 * F, DH, WqT, F, DH, Am, D, (int64_t)NL * D, HEADS, scale},
        {NL, D, DH, KV + F, 2 * F, DH, Wo, F, DH, BtT, D, (int64_t)NL * D, HEADS, 1.0f},
    };
    if ((rc = gemm_group_dispatch(dt, dt, p, 2, fs))) return rc;
  }
  {
    TList t;
    t.add(Am, D, AT, S, S, D, true);         // A [512, 1024] -> AT [1024, 512]
    t.add(BtT, D, Bt, S, S, D, true);        // BtT [512, 1024] -> Bt [1024, 512]
    t.add(latn, D, latnT, NL, NL, D, true);  // [64, 1024] -> [1024, 64]
    if ((rc = launch_tlist<TA, TA>(t, fs))) return rc;
  }
  if (hipEventRecord(side.join, fs) != hipSuccess) {
    set_error("nr_latent_train_step: join 0 record failed");
    return NR_ERR_HIP;
  }
#define NR_LT_TOK(...)                                                       \
  do {                                                                       \
    if (a.tok_dtype == NR_F32) { typedef float TT; __VA_ARGS__; }            \
    else if (a.tok_dtype == NR_BF16) { typedef __bf16 TT; __VA_ARGS__; }     \
    else { typedef _Float16 TT; __VA_ARGS__; }                              \
  } while (0)
  // ---- E[pos] / E[neg] rows for the head (the token LN of those news' last tokens) and their xhat
  NR_LT_TOK(hipLaunchKernelGGL((pn_rows_kernel<TT>), dim3((unsigned)((2 * B + 3) / 4)), dim3(256), 0, st, B,
                               (const TT*)a.tok_last, a.pos, a.neg, a.tok_g, a.tok_b, Epn, Xpn));
  NR_LT_CHECK("pos / neg rows");
  // ---- per-slot forward
  NR_LT_TOK(hipLaunchKernelGGL((gather_ln_kernel<TA, TT>), dim3(grid_rows(Hp)), dim3(256), 0, st, Hp, a.Hs,
                               (const TT*)a.tok_last, a.tok_g, a.tok_b, a.hist_idx, a.nq_g, a.nq_b, 1e-5f, Sx, X));
  NR_LT_CHECK("gather_ln");
  if (hipStreamWaitEvent(st, side.join, 0) != hipSuccess) {
    set_error("nr_latent_train_step: join 0 failed");
    return NR_ERR_HIP;
  }
  if ((rc = gemm_dispatch(dt, dt, NR_EPI_SOFTMAX64, Hp, S, D, X, D, Am, D, nullptr, nullptr, 0, Pm, S, st))) return rc;
  if ((rc = gemm_dispatch(dt, dt, NR_EPI_RESADD, Hp, D, S, Pm, S, Bt, S, nullptr, Sx, D, H1, D, st))) return rc;
  if ((rc = layernorm_dispatch(dt, dt, Hp, D, H1, D, a.nf_g, a.nf_b, 1e-5f, Y, D, st))) return rc;
  if ((rc = gemm_dispatch(dt, dt, NR_EPI_NONE, Hp, 2 * F, D, Y, D, W1, D, a.b1, nullptr, 0, G, 2 * F, st))) return rc;
  // ---- per batch row: means, m = zbar W2^T (split-K) + b2 + h1bar, loss
  hipLaunchKernelGGL((segmean_kernel<TA>), dim3((F + D) / 256, (unsigned)(Bp + 1)), dim3(512), 0, st, B, Bp, a.hist_off, Hp, G,
                     H1, zbar, h1bar, row_seg);
  NR_LT_CHECK("segmean");
  {
    const int64_t ks = F / kHParts;
    GemmProblem p = {Bp, D, ks, zbar, F, ks, W2, F, ks, hparts, D, Bp * D, kHParts, 1.0f};
    if ((rc = gemm_group_dispatch(dt, NR_F32, &p, 1, st))) return rc;
    // the split-K partials summed in parallel (the head reads one row per batch row)
    if ((rc = sum_parts(hparts, kHParts, Bp * D, hsum, Bp * D, st))) return rc;
  }
  hipLaunchKernelGGL((head_kernel<TA>), dim3((unsigned)Bp), dim3(256), 0, st, B, Bp, 1, hsum, a.b2, h1bar,
                     a.hist_off, Epn, a.margin, a.loss, a.users, dmA, dmc, dmc32, Xpn, a.g_tok_g, a.g_tok_b, a.g_b2);
  NR_LT_CHECK("head");
  // ---- backward
  // dZ_b = (dm_b / h_b) W2 (f32, split-K partials [kZParts, Bp, 4096]): C = dmc . W2T^T
  {
    const int64_t ks = D / kZParts;
    GemmProblem p = {Bp, F, ks, dmc, D, ks, W2T, D, ks, dZ, F, Bp * F, kZParts, 1.0f};
    if ((rc = gemm_group_dispatch(dt, NR_F32, &p, 1, st))) return rc;
  }
  if ((rc = sum_parts(dZ, kZParts, Bp * F, dZs, Bp * F, st))) return rc;
  const int64_t gchunks = (Hp + kGRows - 1) / kGRows;
  hipLaunchKernelGGL((geglu_bwd_kernel<TA, kGRows>), dim3(F / 512, (unsigned)gchunks), dim3(256), 0, st, Hp, G, dZs,
                     row_seg, dG, gpart);
  NR_LT_CHECK("geglu_bwd");
  if ((rc = nr_col_sum(NR_F32, gchunks, 2 * F, gpart, 2 * F, a.g_b1, st))) return rc;
  // fork: the weight grads of W1 (K = Hp, 128 tiles) and W2 on the side stream,
  // beside the data-grad GEMM dY = dG W1 (132 persistent workgroups) on this one
  if (hipEventRecord(side.fork, st) != hipSuccess || hipStreamWaitEvent(side.s, side.fork, 0) != hipSuccess) {
    set_error("nr_latent_train_step: fork failed");
    return NR_ERR_HIP;
  }
  if constexpr (sizeof(TA) == 2) {
    // bf16: the weight grads read dG, Y, dm, zbar row-major (TN grouped GEMM, no transposes)
    GemmProblem p[2] = {
        {2 * F, D, Hp, dG, 2 * F, 0, Y, D, 0, a.g_W1, D, 0, 1, 1.0f},
        {D, F, Bp, dmA, D, 0, zbar, F, 0, a.g_W2, F, 0, 1, 1.0f},
    };
    const bool sqf[2] = {true, true};
    if ((rc = gemm_group_tn_dispatch(NR_F32, p, 2, side.s, sqp ? sqp + kSqW12 : nullptr, sqf, &n_sq12,
                                     kSqFold - kSqW12)))
      return rc;
  } else {
    TList t;
    t.add(dG, 2 * F, dGT, Hp, Hp, 2 * F, true);
    t.add(Y, D, YT, Hp, Hp, D, true);
    t.add(dmA, D, dmT, Bp, Bp, D, true);
    t.add(zbar, F, zbarT, Bp, Bp, F, true);
    if ((rc = launch_tlist<TA, TA>(t, side.s))) return rc;
    GemmProblem p[2] = {
        {2 * F, D, Hp, dGT, Hp, 0, YT, Hp, 0, a.g_W1, D, 0, 1, 1.0f},
        {D, F, Bp, dmT, Bp, 0, zbarT, Bp, 0, a.g_W2, F, 0, 1, 1.0f},
    };
    const bool sqf[2] = {true, true};
    if ((rc = gemm_group_dispatch(dt, NR_F32, p, 2, side.s, sqp ? sqp + kSqW12 : nullptr, sqf, &n_sq12,
                                  kSqFold - kSqW12)))
      return rc;
  }
  {
    if (hipEventRecord(side.join, side.s) != hipSuccess) {
      set_error("nr_latent_train_step: join record failed");
      return NR_ERR_HIP;
    }
  }
  if ((rc = gemm_dispatch(dt, dt, NR_EPI_NONE, Hp, D, 2 * F, dG, 2 * F, W1T, 2 * F, nullptr, nullptr, 0, dY, D, st)))
    return rc;
  hipLaunchKernelGGL((ln_bwd_kernel<TA, 0>), dim3(grid_rows(Hp, 512)), dim3(256), 0, st, Hp, Hp, H1, nullptr, a.nf_g, 1e-5f, dY,
                     dmc32, row_seg, dH1, nullptr, nullptr, a.g_nf_g, a.g_nf_b, nullptr, nullptr);
  NR_LT_CHECK("ln_f_bwd");
  if (dt == NR_BF16) {
    // dS = P (dP - sum_group P dP) in the dP GEMM's epilogue (NR_EPI_SOFTMAX64_BWD, R = P)
    if ((rc = gemm_dispatch(dt, dt, NR_EPI_SOFTMAX64_BWD, Hp, S, D, dH1, D, BtT, D, nullptr, Pm, S, dS, S, st)))
      return rc;
  } else {
    if ((rc = gemm_dispatch(dt, dt, NR_EPI_NONE, Hp, S, D, dH1, D, BtT, D, nullptr, nullptr, 0, dP, S, st)))
      return rc;
    const int64_t g = (Hp * HEADS + 3) / 4;
    hipLaunchKernelGGL((softmax64_bwd_kernel<TA>), dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, st, Hp, Pm,
                       dP, dS);
    NR_LT_CHECK("softmax64_bwd");
  }
  // fork 2: dA / dBt and the whole fold backward need only dS, dH1, P, X from here on,
  // so they run on a third stream beside dX and the LN_q / token LN grads.
  // (Starting dBt's transposes and GEMM before the dS GEMM, on a third event, measured
  // no gain: they slowed dS by as much, profiles/round4/train/r4s9.)
  if (hipEventRecord(side.fork2, st) != hipSuccess || hipStreamWaitEvent(side.s2, side.fork2, 0) != hipSuccess) {
    set_error("nr_latent_train_step: fork 2 failed");
    return NR_ERR_HIP;
  }
  if ((rc = gemm_dispatch(dt, dt, NR_EPI_NONE, Hp, D, S, dS, S, AT, S, nullptr, nullptr, 0, dX, D, st))) return rc;
  NR_LT_TOK(hipLaunchKernelGGL((ln_bwd_kernel<TA, 1, TT>), dim3(grid_rows(Hp, 512)), dim3(256), 0, st, Hp, a.Hs, Sx,
                               a.tok_last, a.nq_g, 1e-5f, dX, dH1, a.hist_idx, nullptr, a.g_tok_g, a.g_tok_b,
                               a.g_nq_g, a.g_nq_b, a.tok_g, a.tok_b));
  NR_LT_CHECK("ln_q_bwd");  // (with the head's pos / neg part: the token LN's grads are final)
  {
    // this stream's gradients are all final here
    SqList q;
    const float* gp[] = {a.g_tok_g, a.g_tok_b, a.g_nq_g, a.g_nq_b, a.g_nf_g, a.g_nf_b, a.g_b1, a.g_b2};
    const int64_t gn[] = {D, D, D, D, D, D, 2 * F, D};
    for (int i = 0; i < 8; ++i) q.add(gp[i], gn[i]);
    if ((rc = sq_list(q, a.sumsq, st))) return rc;
  }
  hipStream_t s2 = side.s2;
  // ---- dA = dS^T X and dBt = dH1^T P as kWParts K-slices (16 + 16 tiles alone would hold 32 CUs
  // for a K = Hp tile time), summed while converting to the fold backward's operands
  if constexpr (sizeof(TA) == 2) {
    // bf16: K-slices of the row-major dS / X / dH1 / P (TN grouped GEMM; rows past Hp are zero)
    const int64_t kw = L.kw;
    GemmProblem p[2] = {
        {S, D, kw, dS, S, kw * S, X, D, kw * D, gA, D, (int64_t)S * D, kWParts, 1.0f},
        {D, S, kw, dH1, D, kw * D, Pm, S, kw * S, gBt, S, (int64_t)D * S, kWParts, 1.0f},
    };
    if ((rc = gemm_group_tn_dispatch(NR_F32, p, 2, s2))) return rc;
  } else {
    TList t;
    t.add(dH1, D, dH1T, Hpp, Hp, D, true, Hpp);
    t.add(Pm, S, PT, Hpp, Hp, S, true, Hpp);
    t.add(dS, S, dST, Hpp, Hp, S, true, Hpp);
    t.add(X, D, XT, Hpp, Hp, D, true, Hpp);
    if ((rc = launch_tlist<TA, TA>(t, s2))) return rc;
    const int64_t kw = L.kw;
    GemmProblem p[2] = {
        {S, D, kw, dST, Hpp, kw, XT, Hpp, kw, gA, D, (int64_t)S * D, kWParts, 1.0f},
        {D, S, kw, dH1T, Hpp, kw, PT, Hpp, kw, gBt, S, (int64_t)D * S, kWParts, 1.0f},
    };
    if ((rc = gemm_group_dispatch(dt, NR_F32, p, 2, s2))) return rc;
  }
  // ---- fold backward
  {
    // the K-slices summed on the way into both converted operands (one launch; the
    // slices summed in order)
    SCList t;
    if ((rc = t.add(gA, D, kWParts, (int64_t)S * D, S, D, gA16, D, gAT16, S))) return rc;
    if ((rc = t.add(gBt, S, kWParts, (int64_t)D * S, D, S, gBt16, S, gBtT16, D))) return rc;
    if ((rc = launch_sumconv<TA>(t, s2))) return rc;
  }
  {
    GemmProblem p[4] = {
        // dWq_h [512, 1024] = s K_h^T gA_h: A = KT rows h*512 [512, 64], W = gAT cols h*64 [1024, 64]
        {DH, D, NL, KVT, NL, (int64_t)DH * NL, gAT16, S, NL, a.g_Wq, D, (int64_t)DH * D, HEADS, scale},
        // dK_h [64, 512] = s gA_h Wq_h: A = gA rows h*64 [64, 1024], W = Wq rows h*512 [512, 1024]
        {NL, DH, D, gA16, D, (int64_t)NL * D, Wq, D, (int64_t)DH * D, dKV, 2 * F, DH, HEADS, scale},
        // dV_h [64, 512] = gBtT_h Wo_h: A = gBtT rows h*64 [64, 1024], W = WoT rows h*512 [512, 1024]
        {NL, DH, D, gBtT16, D, (int64_t)NL * D, WoT, D, (int64_t)DH * D, dKV + F, 2 * F, DH, HEADS, 1.0f},
        // dWo_h [1024, 512] = gBt_h V_h: A = gBt cols h*64 [1024, 64], W = VT rows h*512 [512, 64]
        {D, DH, NL, gBt16, S, NL, KVT + (int64_t)F * NL, NL, (int64_t)DH * NL, a.g_Wo, F, DH, HEADS, 1.0f},
    };
    const bool sqf[4] = {true, false, false, true};  // dWq, dWo
    if ((rc = gemm_group_dispatch(dt, NR_F32, p, 4, s2, sqp ? sqp + kSqFold : nullptr, sqf, &n_sqf, kSqKv - kSqFold)))
      return rc;
  }
  {
    SCList t;
    if ((rc = t.add(dKV, 2 * F, 1, 0, NL, 2 * F, dKV16, 2 * F, dKVT16, NL))) return rc;
    if ((rc = launch_sumconv<TA>(t, s2))) return rc;
  }
  {
    const int64_t ks = 2 * F / kLatParts;
    GemmProblem p[2] = {
        // gWkv [8192, 1024] = dKV^T latn: A = dKVT [8192, 64], W = latnT [1024, 64]
        {2 * F, D, NL, dKVT16, NL, 0, latnT, NL, 0, a.g_Wkv, D, 0, 1, 1.0f},
        // dlatn [64, 1024] = dKV Wkv, split-K: A = dKV16 cols, W = WkvT cols
        {NL, D, ks, dKV16, 2 * F, ks, WkvT, 2 * F, ks, dlat, D, (int64_t)NL * D, kLatParts, 1.0f},
    };
    const bool sqf[2] = {true, false};  // dWkv
    if ((rc = gemm_group_dispatch(dt, NR_F32, p, 2, s2, sqp ? sqp + kSqKv : nullptr, sqf, &n_sqkv, kSqSlots - kSqKv)))
      return rc;
  }
  if ((rc = sum_parts(dlat, kLatParts, (int64_t)NL * D, dlat, (int64_t)NL * D, s2))) return rc;
  hipLaunchKernelGGL(lnc_bwd_kernel, dim3(NL / 4), dim3(256), 0, s2, a.latents, a.nc_g, 1e-5f, 1, dlat,
                     a.g_latents, a.g_nc_g, a.g_nc_b);
  NR_LT_CHECK("ln_c_bwd");
  if (hipEventRecord(side.join2, s2) != hipSuccess) {
    set_error("nr_latent_train_step: join 2 record failed");
    return NR_ERR_HIP;
  }
  // join: the side stream's weight grads are done before anything later on `stream`
  if (hipStreamWaitEvent(st, side.join, 0) != hipSuccess || hipStreamWaitEvent(st, side.join2, 0) != hipSuccess) {
    set_error("nr_latent_train_step: join failed");
    return NR_ERR_HIP;
  }
  if (sqp) {
    // the side streams' weight grads: their GEMM-epilogue partials and the squares of
    // the small fold grads (here, not on s2: the optimizer that follows on this stream
    // then starts without a second cross-stream wait)
    SqList q;
    q.add(sqp + kSqW12, n_sq12, false);
    q.add(sqp + kSqFold, n_sqf, false);
    q.add(sqp + kSqKv, n_sqkv, false);
    q.add(a.g_latents, NL * D);
    q.add(a.g_nc_g, D);
    q.add(a.g_nc_b, D);
    if ((rc = sq_list(q, a.sumsq, st))) return rc;
  }
#undef NR_LT_TOK
#undef NR_LT_CHECK
  return NR_OK;
}

}  // namespace lt

// (nr_common.h) one set per host thread and device; the streams are created on
// the device of `st`, so a step launched on another GPU's stream than the
// current device forks and joins on that GPU.
int train_side_streams(hipStream_t st, const char* fn, TrainSide& out) {
  thread_local TrainSide t_side[64];
  int dev = 0;
  if (hipStreamGetDevice(st, &dev) != hipSuccess || dev < 0 || dev >= 64) {
    set_error("%s: cannot resolve the stream's device", fn);
    return NR_ERR_HIP;
  }
  TrainSide& sd = t_side[dev];
  if (!sd.s) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || (cur != dev && hipSetDevice(dev) != hipSuccess)) {
      set_error("%s: cannot select device %d", fn, dev);
      return NR_ERR_HIP;
    }
    const bool ok = hipStreamCreateWithFlags(&sd.s, hipStreamNonBlocking) == hipSuccess &&
                    hipStreamCreateWithFlags(&sd.s2, hipStreamNonBlocking) == hipSuccess &&
                    hipEventCreateWithFlags(&sd.fork, hipEventDisableTiming) == hipSuccess &&
                    hipEventCreateWithFlags(&sd.join, hipEventDisableTiming) == hipSuccess &&
                    hipEventCreateWithFlags(&sd.fork2, hipEventDisableTiming) == hipSuccess &&
                    hipEventCreateWithFlags(&sd.join2, hipEventDisableTiming) == hipSuccess &&
                    hipEventCreateWithFlags(&sd.wt, hipEventDisableTiming) == hipSuccess;
    if (cur != dev) (void)hipSetDevice(cur);
    if (!ok) {
      set_error("%s: cannot create the side streams / events", fn);
      sd = TrainSide{};
      return NR_ERR_HIP;
    }
  }
  out = sd;
  return NR_OK;
}
}  // namespace nr

extern "C" int64_t nr_latent_train_workspace_bytes(int dtype, int64_t B, int64_t U, int64_t Hs) {
  if ((dtype != NR_F32 && dtype != NR_BF16) || B < 0 || U < 0 || Hs < 0) return -1;
  return nr::lt::layout(dtype, B, U, Hs).total;
}

extern "C" int nr_latent_train_step(const nr_latent_train_args* args, void* ws, int64_t ws_bytes, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(args, "nr_latent_train_step: null args");
  const nr_latent_train_args& a = *args;
  NR_CHECK_ARG(a.dtype == NR_F32 || a.dtype == NR_BF16, "nr_latent_train_step: dtype must be NR_F32 or NR_BF16");
  NR_CHECK_ARG(a.tok_dtype == NR_F32 || a.tok_dtype == NR_BF16 || a.tok_dtype == NR_F16,
               "nr_latent_train_step: bad tok_dtype");
  NR_CHECK_ARG(a.B >= 1 && a.U >= 1 && a.Hs >= 1, "nr_latent_train_step: empty batch (B=%lld U=%lld Hs=%lld)",
               (long long)a.B, (long long)a.U, (long long)a.Hs);
  NR_CHECK_ARG(a.Hs <= (1ll << 31) - 1024 && a.U <= (1ll << 31) && a.B <= (1ll << 24),
               "nr_latent_train_step: batch too large");
  NR_CHECK_DEVICE("nr_latent_train_step", a.tok_last, a.hist_idx, a.hist_off, a.pos, a.neg, a.tok_g, a.tok_b,
                  a.latents, a.nq_g, a.nq_b, a.nc_g, a.nc_b, a.Wq, a.Wkv, a.Wo, a.nf_g, a.nf_b, a.W1, a.b1, a.W2, a.b2);
  NR_CHECK_DEVICE("nr_latent_train_step", a.g_tok_g, a.g_tok_b, a.g_latents, a.g_nq_g, a.g_nq_b, a.g_nc_g, a.g_nc_b,
                  a.g_Wq, a.g_Wkv, a.g_Wo, a.g_nf_g, a.g_nf_b, a.g_W1, a.g_b1, a.g_W2, a.g_b2, a.loss, a.users, a.sumsq,
                  ws);
  NR_CHECK_ARG(a.tok_last && a.hist_idx && a.hist_off && a.pos && a.neg && a.loss && ws,
               "nr_latent_train_step: null pointer");
  const int64_t need = nr::lt::layout(a.dtype, a.B, a.U, a.Hs).total;
  NR_CHECK_ARG(ws_bytes >= need, "nr_latent_train_step: workspace too small (%lld < %lld)", (long long)ws_bytes,
               (long long)need);
  NR_CHECK_ARG(((uintptr_t)ws & 255) == 0, "nr_latent_train_step: workspace must be 256-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  return a.dtype == NR_F32 ? nr::lt::step<float>(a, (char*)ws, s) : nr::lt::step<__bf16>(a, (char*)ws, s);
}
