// Training-step kernels of config 5 (reference scripts/train_v3.py ->
// AttentionAttentionTrainer.train_one_epoch, trainer.py:1030-1117):
//   token model (g_mlp_layernorm of the last valid token) -> history gather ->
//   FinalAttention per valid history slot (GEMMs in gemm.hip, dropout fused in
//   the ReLU epilogue) -> per-dimension softmax pooling -> cosine vs the
//   positive / negative news -> MarginRankingLoss(2) -> backward ->
//   clip_grad_norm_(0.5) -> AdamW.
// The GEMMs (forward, data-grad and weight-grad) all run on the C = A·Wᵀ MFMA
// kernel; the weight-grad and data-grad operands are produced by the LDS
// transpose below.  Everything here is HBM-bound row / reduction work.
#include "nr_common.h"

namespace nr {

template <typename T>
__device__ __forceinline__ float ldf(const T* p) {
  if constexpr (sizeof(T) == 4) return *p; else return (float)*p;
}
template <typename T>
__device__ __forceinline__ void stf(T* p, float v) {
  if constexpr (sizeof(T) == 4) *p = v; else *p = (T)v;
}

// ----------------------------------------------------------------- gather rows
// dst[i] = src[idx[i]] (idx < 0 -> zero row), with dtype conversion.
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void gather_rows_kernel(int64_t n, int64_t dim, const TI* __restrict__ src,
                                                          int64_t lds, const int32_t* __restrict__ idx,
                                                          TO* __restrict__ dst, int64_t ldd) {
  const int64_t i = (int64_t)blockIdx.x;
  if (i >= n) return;
  const int64_t r = idx ? idx[i] : i;
  for (int64_t c = threadIdx.x; c < dim; c += 256) stf<TO>(dst + i * ldd + c, r < 0 ? 0.f : ldf<TI>(src + r * lds + c));
}

// ----------------------------------------------------------------- transpose
// dst[c][r] = src[r][c] through a 64x65 f32 LDS tile (256 threads).
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void transpose_kernel(int64_t rows, int64_t cols, const TI* __restrict__ src,
                                                        int64_t lds, TO* __restrict__ dst, int64_t ldd) {
  __shared__ float tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int rr = ty + 4 * k;
    const int64_t r = r0 + rr, c = c0 + tx;
    tile[rr][tx] = (r < rows && c < cols) ? ldf<TI>(src + r * lds + c) : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int cc = ty + 4 * k;
    const int64_t c = c0 + cc, r = r0 + tx;
    if (c < cols && r < rows) stf<TO>(dst + c * ldd + r, tile[tx][cc]);
  }
}

// 16-bit -> 16-bit transpose of a 64x64 tile with 16-B global accesses: each
// lane loads 8 consecutive columns of a row (2 per lane), the tile sits in LDS
// as u16 rows of pitch 66 (odd dword pitch: the column reads below are at most
// 2-way), and each lane writes 8 consecutive source rows of one column as one
// 16-B store (8 lanes = one 128-B output row segment).  Needs rows, cols,
// strides multiple of 8 and 16-B aligned bases (checked by the caller).
__global__ __launch_bounds__(256) void transpose16_kernel(int64_t rows, int64_t cols,
                                                          const uint16_t* __restrict__ src, int64_t lds,
                                                          uint16_t* __restrict__ dst, int64_t ldd) {
  constexpr int P = 66;
  __shared__ uint16_t tile[64 * P];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int rr = (t >> 3) + 32 * k, ch = t & 7;
    const int64_t r = r0 + rr, c = c0 + 8 * ch;
    uint4 u = make_uint4(0, 0, 0, 0);
    if (r < rows && c < cols) u = *reinterpret_cast<const uint4*>(src + r * lds + c);
    uint32_t* d = reinterpret_cast<uint32_t*>(tile + rr * P + 8 * ch);  // 4-B aligned (P even)
    d[0] = u.x; d[1] = u.y; d[2] = u.z; d[3] = u.w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int oc = (t >> 3) + 32 * k, rc = t & 7;
    const int64_t c = c0 + oc, r = r0 + 8 * rc;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)tile[(8 * rc + 2 * j) * P + oc] | ((uint32_t)tile[(8 * rc + 2 * j + 1) * P + oc] << 16);
    if (c < cols && r < rows) *reinterpret_cast<uint4*>(dst + c * ldd + r) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// f32 -> bf16 transpose of a 64x64 tile with 16-B global accesses both ways
// (the generic kernel above stores 2 B per lane): 16 lanes load one source
// row as float4s into a 64x65 f32 LDS tile (rr + 4ch distinct mod 64: no bank
// conflict), then each lane converts 8 consecutive source rows of one column
// (8rc + oc distinct mod 64) and writes them as one 16-B store.  Same (__bf16)
// rounding as the generic kernel, so the result is bit-identical.  Needs rows,
// ldd multiples of 8, cols, lds multiples of 4 and 16-B aligned bases.
__global__ __launch_bounds__(256) void transpose_f32_bf16_kernel(int64_t rows, int64_t cols,
                                                                 const float* __restrict__ src, int64_t lds,
                                                                 __bf16* __restrict__ dst, int64_t ldd) {
  __shared__ float tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int rr = (t >> 4) + 16 * k, ch = t & 15;
    const int64_t r = r0 + rr, c = c0 + 4 * ch;
    float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < rows && c < cols) u = *reinterpret_cast<const float4*>(src + r * lds + c);
    tile[rr][4 * ch] = u.x; tile[rr][4 * ch + 1] = u.y; tile[rr][4 * ch + 2] = u.z; tile[rr][4 * ch + 3] = u.w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int oc = (t >> 3) + 32 * k, rc = t & 7;
    const int64_t c = c0 + oc, r = r0 + 8 * rc;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = __builtin_bit_cast(uint16_t, (__bf16)tile[8 * rc + 2 * j][oc]);
      const uint32_t hi = __builtin_bit_cast(uint16_t, (__bf16)tile[8 * rc + 2 * j + 1][oc]);
      w[j] = lo | (hi << 16);
    }
    if (c < cols && r < rows) *reinterpret_cast<uint4*>(dst + c * ldd + r) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// ----------------------------------------------------------------- pooling fwd
// FinalAttention pooling (modeling_utils.py:224-228) over consecutive slot rows:
// xp row = [x | p] (p = exp(w)); u_d = sum x p / (sum p + 1e-10), z_d = sum p + 1e-10.
// One workgroup (4 waves x 256 dims) per segment.
// 4 consecutive elements as one 8-B (bf16) / 16-B (f32) access (host: 16-B aligned
// base, row strides and column offsets multiples of 4 elements)
template <typename T>
__device__ __forceinline__ void ld4v(const T* p, float (&v)[4]) {
  if constexpr (sizeof(T) == 4) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    const uint2 q = *reinterpret_cast<const uint2*>(p);
    v[0] = bf16_lo(q.x); v[1] = bf16_hi(q.x); v[2] = bf16_lo(q.y); v[3] = bf16_hi(q.y);
  }
}
template <typename T>
__device__ __forceinline__ void st4v(T* p, const float (&v)[4]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
  } else {
    const __bf16 h[4] = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(h);
  }
}

// ----------------------------------------------------------------- pooling fwd
// u[b, d] = sum_i x[i, d] p[i, d] / (sum_i p[i, d] + 1e-10) over the rows of
// segment b (FinalAttention's per-dimension softmax pooling, modeling_utils.py:224-228,
// with p = exp(logit) from the GEMM epilogue); z = the denominator (saved for bwd).
// Block = (segment, 256-dim quarter) with kPoolWaves waves striding the segment's
// rows (4 dims per lane, one 8-B load of x and of p per row), partial sums folded
// through LDS in a fixed order.  16 waves: the history lengths are geometric up to
// 600 and the longest segment's block sets the kernel time (4 waves: 26 us).
constexpr int kPoolWaves = 16;
template <typename T>
__global__ __launch_bounds__(64 * kPoolWaves) void final_pool_fwd_kernel(int64_t n_seg, const int64_t* __restrict__ off,
                                                                        const T* __restrict__ xp, int64_t ld,
                                                                        float* __restrict__ users,
                                                                        float* __restrict__ z) {
  constexpr int D = 1024;
  __shared__ float sn[kPoolWaves][256], sd[kPoolWaves][256];
  const int64_t b = blockIdx.x;
  if (b >= n_seg) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int d = (int)blockIdx.y * 256 + lane * 4;
  float num[4] = {0.f, 0.f, 0.f, 0.f}, den[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int64_t i = off[b] + wave; i < off[b + 1]; i += kPoolWaves) {
    const T* row = xp + i * ld;
    float x[4], p[4];
    ld4v<T>(row + d, x);
    ld4v<T>(row + D + d, p);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      num[t] = fmaf(x[t], p[t], num[t]);
      den[t] += p[t];
    }
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) { sn[wave][lane * 4 + t] = num[t]; sd[wave][lane * 4 + t] = den[t]; }
  __syncthreads();
  if (threadIdx.x < 256) {
    const int c = threadIdx.x, dc = (int)blockIdx.y * 256 + c;
    float sdn = 0.f, snn = 0.f;
#pragma unroll
    for (int w = 0; w < kPoolWaves; ++w) { sdn += sd[w][c]; snn += sn[w][c]; }
    const float zz = sdn + 1e-10f;
    z[b * D + dc] = zz;
    users[b * D + dc] = snn / zz;
  }
}

// ----------------------------------------------------------------- pooling bwd
// dx_i = du * p_i / z ;  dlogit_i = du * (x_i - u) / z * p_i  (d p_i / d w_i = p_i).
// Rows of no segment (padding up to n_rows) get zeros.  Every row is independent
// given its segment's (du, u, z), so the grid runs over ROWS, not segments: block =
// 16 rows x one 256-dim quarter, wave w rows 4 w .. 4 w + 3, 4 dims per lane, the
// row's segment found by a binary search of off for the wave's first row and
// stepped after (rows are in segment order).  Per-segment blocks waited on the
// longest history (geometric lengths up to 600): 31 us at 4 waves, 22 at 16.
template <typename T>
__global__ __launch_bounds__(256) void final_pool_bwd_kernel(int64_t n_seg, const int64_t* __restrict__ off,
                                                             int64_t n_rows, const T* __restrict__ xp, int64_t ld,
                                                             const float* __restrict__ users,
                                                             const float* __restrict__ z,
                                                             const float* __restrict__ du, T* __restrict__ dx,
                                                             int64_t lddx, T* __restrict__ dl, int64_t lddl) {
  constexpr int D = 1024;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int d = (int)blockIdx.y * 256 + lane * 4;
  const int64_t r0 = (int64_t)blockIdx.x * 16 + wave * 4;
  const int64_t nvalid = off[n_seg];
  int64_t b = -1, bend = 0;  // current segment and its end row
  float g[4], u[4], iz[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t i = r0 + k;
    if (i >= n_rows) break;
    if (i >= nvalid) {
      const float zero[4] = {0.f, 0.f, 0.f, 0.f};
      st4v<T>(dx + i * lddx + d, zero);
      st4v<T>(dl + i * lddl + d, zero);
      continue;
    }
    if (i >= bend) {
      if (b < 0) {  // largest b with off[b] <= i (off[0] = 0 <= i < off[n_seg])
        int64_t lo = 0, hi = n_seg - 1;
        while (lo < hi) {
          const int64_t mid = (lo + hi + 1) >> 1;
          if (off[mid] <= i) lo = mid; else hi = mid - 1;
        }
        b = lo;
      } else {
        do { ++b; } while (off[b + 1] <= i);  // (empty segments are stepped over)
      }
      bend = off[b + 1];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        g[t] = du[b * D + d + t];
        u[t] = users[b * D + d + t];
        iz[t] = 1.0f / z[b * D + d + t];
      }
    }
    const T* row = xp + i * ld;
    float x[4], p[4], gx[4], gl[4];
    ld4v<T>(row + d, x);
    ld4v<T>(row + D + d, p);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      gx[t] = g[t] * p[t] * iz[t];
      gl[t] = gx[t] * (x[t] - u[t]);
    }
    st4v<T>(dx + i * lddx + d, gx);
    st4v<T>(dl + i * lddl + d, gl);
  }
}

// ----------------------------------------------------------------- cosine + margin loss
// F.cosine_similarity(u, e) = (u / max(|u|, 1e-8)) . (e / max(|e|, 1e-8))
// (data_model_helper.py / trainer.py:1058-1061), MarginRankingLoss(margin)(s_pos,
// s_neg, y=1) = mean(clamp_min(margin - (s_pos - s_neg), 0)) (trainer.py:1063-1066).
// One wave per batch row; du written, dE rows (pos / neg) accumulated with atomics.
__global__ __launch_bounds__(256) void cosine_margin_kernel(int64_t B, const float* __restrict__ users,
                                                            const float* __restrict__ E, int64_t lde,
                                                            const int32_t* __restrict__ pos,
                                                            const int32_t* __restrict__ neg, float margin,
                                                            float* __restrict__ s_out, float* __restrict__ loss,
                                                            float* __restrict__ du, float* __restrict__ dE) {
  constexpr int D = 1024, NJ = D / 256;
  constexpr float EPS = 1e-8f;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float u[NJ][4], ep[NJ][4], en[NJ][4];
  float uu = 0.f, pp = 0.f, nn = 0.f, up = 0.f, un = 0.f;
  const float* ur = users + b * D;
  const float* pr = E + (int64_t)pos[b] * lde;
  const float* nr_ = E + (int64_t)neg[b] * lde;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int e = j * 256 + lane * 4;
    const float4 a = *reinterpret_cast<const float4*>(ur + e);
    const float4 p = *reinterpret_cast<const float4*>(pr + e);
    const float4 q = *reinterpret_cast<const float4*>(nr_ + e);
    u[j][0] = a.x; u[j][1] = a.y; u[j][2] = a.z; u[j][3] = a.w;
    ep[j][0] = p.x; ep[j][1] = p.y; ep[j][2] = p.z; ep[j][3] = p.w;
    en[j][0] = q.x; en[j][1] = q.y; en[j][2] = q.z; en[j][3] = q.w;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      uu = fmaf(u[j][t], u[j][t], uu);
      pp = fmaf(ep[j][t], ep[j][t], pp);
      nn = fmaf(en[j][t], en[j][t], nn);
      up = fmaf(u[j][t], ep[j][t], up);
      un = fmaf(u[j][t], en[j][t], un);
    }
  }
  uu = wave_sum(uu); pp = wave_sum(pp); nn = wave_sum(nn); up = wave_sum(up); un = wave_sum(un);
  const float nu = sqrtf(uu), np_ = sqrtf(pp), nq = sqrtf(nn);
  const float iu = 1.0f / fmaxf(nu, EPS), ip = 1.0f / fmaxf(np_, EPS), iq = 1.0f / fmaxf(nq, EPS);
  const float sp = up * iu * ip, sn = un * iu * iq;
  const float v = margin - (sp - sn);
  const float act = v >= 0.f ? 1.0f : 0.0f;  // clamp_min backward passes where input >= min
  const float gsp = -act / (float)B, gsn = act / (float)B;
  if (lane == 0) {
    if (s_out) { s_out[b] = sp; s_out[B + b] = sn; }
    atomicAdd(loss, fmaxf(v, 0.f) / (float)B);
  }
  // d cos(u, e) / du = (ê - [|u| > eps] cos û) / max(|u|, eps)   (û = u / max(|u|, eps))
  const float cu = nu > EPS ? 1.f : 0.f, cp = np_ > EPS ? 1.f : 0.f, cq = nq > EPS ? 1.f : 0.f;
  float* dp = dE + (int64_t)pos[b] * lde;
  float* dn = dE + (int64_t)neg[b] * lde;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int e = j * 256 + lane * 4;
    float g[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float uh = u[j][t] * iu, ph = ep[j][t] * ip, qh = en[j][t] * iq;
      g[t] = gsp * (ph - cu * sp * uh) * iu + gsn * (qh - cu * sn * uh) * iu;
      atomicAdd(dp + e + t, gsp * (uh - cp * sp * ph) * ip);
      atomicAdd(dn + e + t, gsn * (uh - cq * sn * qh) * iq);
    }
    *reinterpret_cast<float4*>(du + b * D + e) = make_float4(g[0], g[1], g[2], g[3]);
  }
}

// ----------------------------------------------------------------- scatter add
template <typename T>
__global__ __launch_bounds__(256) void scatter_add_rows_kernel(int64_t n, int64_t dim, const T* __restrict__ src,
                                                               int64_t lds, const int32_t* __restrict__ idx,
                                                               float* __restrict__ dst, int64_t ldd) {
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const int32_t r = idx[i];
  if (r < 0) return;
  for (int64_t c = threadIdx.x; c < dim; c += 256) atomicAdd(dst + (int64_t)r * ldd + c, ldf<T>(src + i * lds + c));
}

// ----------------------------------------------------------------- column sums
// out[c] += sum_r src[r][c]; 64 rows x 256 columns per workgroup, atomics per column.
template <typename T>
__global__ __launch_bounds__(256) void col_sum_kernel(int64_t rows, int64_t cols, const T* __restrict__ src,
                                                      int64_t lds, int rows_per_block, float* __restrict__ out) {
  // block = 512 columns (8 per lane, one 16-B (bf16) / 2x16-B (f32) load per
  // row) x rows_per_block rows, the 4 waves striding the rows; partials
  // folded in LDS, then one atomic per column per block.
  __shared__ float part[4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 512 + lane * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float s[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = 0.f;
  const bool vec = c + 8 <= cols && (lds % 8) == 0 && ((uintptr_t)src & 15) == 0;
  if (vec) {
    for (int64_t r = r0 + wave; r < r1; r += 4) {
      const T* p = src + r * lds + c;
      if constexpr (sizeof(T) == 2) {
        const uint4 u = *reinterpret_cast<const uint4*>(p);
        const T* h = reinterpret_cast<const T*>(&u);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += (float)h[e];
      } else {
        const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
        s[0] += a.x; s[1] += a.y; s[2] += a.z; s[3] += a.w;
        s[4] += b.x; s[5] += b.y; s[6] += b.z; s[7] += b.w;
      }
    }
  } else if (c < cols) {
    for (int64_t r = r0 + wave; r < r1; r += 4)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c + e < cols) s[e] += ldf<T>(src + r * lds + c + e);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[wave][lane * 8 + e] = s[e];
  __syncthreads();
  for (int j = threadIdx.x; j < 512; j += 256) {
    const int64_t cc = (int64_t)blockIdx.x * 512 + j;
    if (cc < cols) atomicAdd(out + cc, (part[0][j] + part[1][j]) + (part[2][j] + part[3][j]));
  }
}

// ----------------------------------------------------------------- LN param grads
// E = LN(x) * g + b  ->  dg += dE * xhat, db += dE (rows gathered by row_idx).
// One wave per row; per-row partials folded into per-block LDS sums first.
template <typename TI>
__global__ __launch_bounds__(256) void ln_param_grad_kernel(int64_t n, const TI* __restrict__ x, int64_t ldx,
                                                            const int64_t* __restrict__ row_idx, float eps,
                                                            const float* __restrict__ dy, int64_t lddy,
                                                            float* __restrict__ dg, float* __restrict__ db) {
  constexpr int D = 1024, NJ = D / 256;
  // per-lane register accumulators for the lane's 16 columns (no LDS atomics)
  __shared__ float sg[4][D], sb[4][D];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float ag[NJ][4], ab[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) { ag[j][t] = 0.f; ab[j][t] = 0.f; }
  for (int64_t i = (int64_t)blockIdx.x * 4 + wave; i < n; i += (int64_t)gridDim.x * 4) {
    const int64_t row = row_idx ? row_idx[i] : i;
    float v[NJ][4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v[j][t] = ldf<TI>(x + row * ldx + j * 256 + lane * 4 + t);
        s += v[j][t];
      }
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) { const float dd = v[j][t] - mean; q = fmaf(dd, dd, q); }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float4 g = *reinterpret_cast<const float4*>(dy + i * lddy + j * 256 + lane * 4);
      const float gg[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        ag[j][t] = fmaf(gg[t], (v[j][t] - mean) * rstd, ag[j][t]);
        ab[j][t] += gg[t];
      }
    }
  }
  // fold the 4 waves' register partials in LDS (fixed order), one atomic per column per block
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sg[wave][j * 256 + lane * 4 + t] = ag[j][t];
      sb[wave][j * 256 + lane * 4 + t] = ab[j][t];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    atomicAdd(dg + c, (sg[0][c] + sg[1][c]) + (sg[2][c] + sg[3][c]));
    atomicAdd(db + c, (sb[0][c] + sb[1][c]) + (sb[2][c] + sb[3][c]));
  }
}

// ----------------------------------------------------------------- latent attention training (f32)
// Per-item pieces of LatentAttentionModel's backward (latent_attention.py:157-163):
// PreNorm LayerNorm input gradient, the per-head softmax (64 latents) backward,
// and GEGLU forward / backward (x, gates = chunk(2); x * gelu(gates), exact erf).

// dx = rstd (dxh - mean(dxh) - xhat mean(dxh xhat)) + dres,  dxh = dy * gamma;
// one wave per row (D = 1024, 16 columns per lane), stats recomputed from x
// with the forward's two-pass arithmetic.  dres may alias dx (in place).
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(int64_t n, const float* __restrict__ x, int64_t ldx,
                                                            const float* __restrict__ gamma, float eps,
                                                            const float* __restrict__ dy, int64_t lddy,
                                                            const float* dres, int64_t ldr, float* dx,
                                                            int64_t lddx) {
  constexpr int D = 1024, NJ = D / 256;
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += (int64_t)gridDim.x * 4) {
    float v[NJ][4], g[NJ][4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float4 a = *reinterpret_cast<const float4*>(x + row * ldx + j * 256 + lane * 4);
      v[j][0] = a.x; v[j][1] = a.y; v[j][2] = a.z; v[j][3] = a.w;
      s += (a.x + a.y) + (a.z + a.w);
    }
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) { const float d = v[j][t] - mean; q = fmaf(d, d, q); }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float4 d4 = *reinterpret_cast<const float4*>(dy + row * lddy + j * 256 + lane * 4);
      const float4 g4 = gamma ? *reinterpret_cast<const float4*>(gamma + j * 256 + lane * 4)
                              : float4{1.f, 1.f, 1.f, 1.f};
      const float dd[4] = {d4.x, d4.y, d4.z, d4.w}, gg[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v[j][t] = (v[j][t] - mean) * rstd;  // xhat
        g[j][t] = dd[t] * gg[t];            // dxhat
        s1 += g[j][t];
        s2 = fmaf(g[j][t], v[j][t], s2);
      }
    }
    const float m1 = wave_sum(s1) / (float)D, m2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float o[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = rstd * (g[j][t] - m1 - v[j][t] * m2);
      if (dres) {
        const float4 r4 = *reinterpret_cast<const float4*>(dres + row * ldr + j * 256 + lane * 4);
        o[0] += r4.x; o[1] += r4.y; o[2] += r4.z; o[3] += r4.w;
      }
      *reinterpret_cast<float4*>(dx + row * lddx + j * 256 + lane * 4) = float4{o[0], o[1], o[2], o[3]};
    }
  }
}

// dS = P * (dP - sum_group(P * dP)) over groups of 64 columns (one head's
// latents; SDPA softmax, latent_attention.py:72).  One wave per (row, group).
template <typename TO>
__global__ __launch_bounds__(256) void softmax64_bwd_kernel(int64_t n_groups, int64_t groups_per_row,
                                                            const float* __restrict__ p, int64_t ldp,
                                                            const float* __restrict__ dp, int64_t lddp,
                                                            TO* __restrict__ ds, int64_t ldds) {
  const int lane = threadIdx.x & 63;
  for (int64_t gi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); gi < n_groups; gi += (int64_t)gridDim.x * 4) {
    const int64_t row = gi / groups_per_row, col = (gi % groups_per_row) * 64 + lane;
    const float pv = p[row * ldp + col], dv = dp[row * lddp + col];
    const float dot = wave_sum(pv * dv);
    stf<TO>(ds + row * ldds + col, pv * (dv - dot));
  }
}

__device__ __forceinline__ float gelu_exact(float g) { return 0.5f * g * (1.0f + erff(g * 0.70710678118654752440f)); }

// z[:, j] = a_j * gelu(g_j),  a = G[:, :F], g = G[:, F:]  (GEGLU, latent_attention.py:24-27)
template <typename TO>
__device__ __forceinline__ void st4(TO* p, float a, float b, float c, float d) {
  if constexpr (sizeof(TO) == 4) {
    *reinterpret_cast<float4*>(p) = float4{a, b, c, d};
  } else {
    p[0] = (TO)a; p[1] = (TO)b; p[2] = (TO)c; p[3] = (TO)d;
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void geglu_fwd_kernel(int64_t rows, int64_t f, const float* __restrict__ G,
                                                        int64_t ldg, TO* __restrict__ z, int64_t ldz) {
  const int64_t total = rows * f;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < total; i += (int64_t)gridDim.x * 1024) {
    const int64_t r = i / f, c = i % f;  // f % 4 == 0: the 4 columns share a row
    const float4 a = *reinterpret_cast<const float4*>(G + r * ldg + c);
    const float4 g = *reinterpret_cast<const float4*>(G + r * ldg + f + c);
    st4<TO>(z + r * ldz + c, a.x * gelu_exact(g.x), a.y * gelu_exact(g.y), a.z * gelu_exact(g.z),
            a.w * gelu_exact(g.w));
  }
}

// dG[:, j] = dz_j gelu(g_j);  dG[:, F + j] = dz_j a_j gelu'(g_j),
// gelu'(g) = Phi(g) + g phi(g)  (the derivative torch's gelu backward uses)
template <typename TO>
__global__ __launch_bounds__(256) void geglu_bwd_kernel(int64_t rows, int64_t f, const float* __restrict__ G,
                                                        int64_t ldg, const float* __restrict__ dz, int64_t lddz,
                                                        TO* __restrict__ dG, int64_t lddg) {
  const int64_t total = rows * f;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < total; i += (int64_t)gridDim.x * 1024) {
    const int64_t r = i / f, c = i % f;
    const float4 a4 = *reinterpret_cast<const float4*>(G + r * ldg + c);
    const float4 g4 = *reinterpret_cast<const float4*>(G + r * ldg + f + c);
    const float4 d4 = *reinterpret_cast<const float4*>(dz + r * lddz + c);
    const float a[4] = {a4.x, a4.y, a4.z, a4.w}, g[4] = {g4.x, g4.y, g4.z, g4.w}, d[4] = {d4.x, d4.y, d4.z, d4.w};
    float da[4], dg[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float cdf = 0.5f * (1.0f + erff(g[t] * 0.70710678118654752440f));
      const float pdf = 0.39894228040143267794f * expf(-0.5f * g[t] * g[t]);
      da[t] = d[t] * g[t] * cdf;
      dg[t] = d[t] * a[t] * (cdf + g[t] * pdf);
    }
    st4<TO>(dG + r * lddg + c, da[0], da[1], da[2], da[3]);
    st4<TO>(dG + r * lddg + f + c, dg[0], dg[1], dg[2], dg[3]);
  }
}

// ----------------------------------------------------------------- grad norm + AdamW
// Sum of squares: 16-B lane loads, grid-stride over <= 1024 blocks, block
// reduction in LDS, ONE atomic per block (per-wave atomics on a single address
// serialise at the memory side: MI355X_MICROARCH.md "Global float atomics").
__global__ __launch_bounds__(256) void sumsq_kernel(int64_t n, const float* __restrict__ x, float* __restrict__ out) {
  __shared__ float part[4];
  float s = 0.f;
  const int64_t n4 = ((uintptr_t)x & 15) == 0 ? n / 4 : 0;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  // four 16-B loads in flight per thread (one per iteration left the kernel
  // latency-bound: 30 us for the latent step's 114 MB of gradients)
  const int64_t gs = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
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
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    s = fmaf(x[i], x[i], s);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (part[0] + part[1]) + (part[2] + part[3]));
}

// torch.nn.utils.clip_grad_norm_(max_norm): coef = min(max_norm / (norm + 1e-6), 1)
// torch.optim.AdamW (weight decay decoupled, bias-corrected):
//   p *= 1 - lr wd;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
__device__ __forceinline__ void adamw_one(float& p, float g, float& m, float& v, float lr, float b1, float b2,
                                          float eps, float wd, float bc1, float bc2s) {
  p *= 1.f - lr * wd;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  p -= (lr / bc1) * m / (sqrtf(v) / bc2s + eps);
}

// 4 parameters per lane (16-B loads / stores of p, g, m, v; 8-B bf16 mirror
// store) when every array is aligned for it, scalar tail / fallback otherwise.
__global__ __launch_bounds__(256) void adamw_kernel(int64_t n, float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    __bf16* __restrict__ p16, float lr, float b1, float b2,
                                                    float eps, float wd, float bc1, float bc2s, float max_norm,
                                                    const float* __restrict__ sumsq) {
  float coef = 1.f;
  if (sumsq) coef = fminf(max_norm / (sqrtf(*sumsq) + 1e-6f), 1.f);
  const bool vec = ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0) &&
                   (((uintptr_t)p16 & 7) == 0);
  const int64_t n4 = vec ? n / 4 : 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    adamw_one(pp.x, gg.x * coef, mm.x, vv.x, lr, b1, b2, eps, wd, bc1, bc2s);
    adamw_one(pp.y, gg.y * coef, mm.y, vv.y, lr, b1, b2, eps, wd, bc1, bc2s);
    adamw_one(pp.z, gg.z * coef, mm.z, vv.z, lr, b1, b2, eps, wd, bc1, bc2s);
    adamw_one(pp.w, gg.w * coef, mm.w, vv.w, lr, b1, b2, eps, wd, bc1, bc2s);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (p16) {
      __bf16 h[4] = {(__bf16)pp.x, (__bf16)pp.y, (__bf16)pp.z, (__bf16)pp.w};
      *reinterpret_cast<uint2*>(p16 + 4 * i) = *reinterpret_cast<const uint2*>(h);
    }
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_one(pi, g[i] * coef, mi, vi, lr, b1, b2, eps, wd, bc1, bc2s);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (p16) p16[i] = (__bf16)pi;
  }
}

static int grid_for(int64_t n) { const int64_t g = (n + 255) / 256; return (int)(g < 4096 ? g : 4096); }

}  // namespace nr

using namespace nr;

#define NR_DT2(dti, dto, ...)                                                              \
  do {                                                                                     \
    if (dti == NR_F32 && dto == NR_F32) { typedef float TI; typedef float TO; __VA_ARGS__; } \
    else if (dti == NR_F32) { typedef float TI; typedef __bf16 TO; __VA_ARGS__; }           \
    else if (dto == NR_F32) { typedef __bf16 TI; typedef float TO; __VA_ARGS__; }           \
    else { typedef __bf16 TI; typedef __bf16 TO; __VA_ARGS__; }                            \
  } while (0)
// ----------------------------------------------------------------- split-K fixup
// C[r][c] = epi(sum_s P[s][r][c] + bias[c]) for the rows of a GEMM that were
// computed as `parts` K-slices (nr_gemm_grouped, f32 partials), with the
// epilogues of the training GEMMs: ReLU + dropout (same counter-hash mask as
// the GEMM kernels: drop_at(seed, (row0 + r) * N + c, thr)) and the relu/dropout
// backward (R > 0 ? v * scale : 0).  4 columns per thread.
template <int EPI, typename TO>
__global__ __launch_bounds__(256) void splitk_fixup_kernel(int64_t rows, int64_t N, int parts, const float* __restrict__ P,
                                                           const float* __restrict__ bias, const TO* __restrict__ R,
                                                           int64_t ldr, TO* __restrict__ C, int64_t ldc, int64_t row0,
                                                           uint64_t seed, uint32_t thr, float scale) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // quad index
  const int64_t nq = N / 4;
  if (q >= rows * nq) return;
  const int64_t r = q / nq, c = (q % nq) * 4;
  f32x4 v = *reinterpret_cast<const f32x4*>(P + r * N + c);
  for (int s = 1; s < parts; ++s) v += *reinterpret_cast<const f32x4*>(P + ((int64_t)s * rows + r) * N + c);
  uint64_t dh = 0;  // c % 4 == 0: the 4 columns are one group of the dropout stream
  if constexpr (EPI == NR_EPI_RELU_DROPOUT) dh = drop_hash4(seed, (uint64_t)((row0 + r) * N + c) >> 2);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float x = v[k] + (bias ? bias[c + k] : 0.f);
    if constexpr (EPI == NR_EPI_RELU_DROPOUT) x = drop_field(dh, k, thr) ? 0.f : fmaxf(x, 0.f) * scale;
    if constexpr (EPI == NR_EPI_DRELU) x = ldf(R + r * ldr + c + k) > 0.f ? x * scale : 0.f;
    if constexpr (EPI == NR_EPI_RESADD) x += ldf(R + r * ldr + c + k);
    if constexpr (EPI == NR_EPI_EXP) x = __expf(x);  // as the bf16 GEMM epilogue (gemm.hip epi_exp)
    stf(C + r * ldc + c + k, x);
  }
}

#define NR_DT1(dt, ...)                                       \
  do {                                                        \
    if (dt == NR_F32) { typedef float T; __VA_ARGS__; }       \
    else { typedef __bf16 T; __VA_ARGS__; }                   \
  } while (0)
#define NR_OKDT(d) ((d) == NR_F32 || (d) == NR_BF16)

extern "C" int nr_gather_rows(int dtype_in, int dtype_out, int64_t n, int64_t dim, const void* src, int64_t lds,
                              const int32_t* idx, void* dst, int64_t ldd, void* stream) {
  clear_error();
  NR_CHECK_ARG(NR_OKDT(dtype_in) && NR_OKDT(dtype_out), "nr_gather_rows: bad dtype");
  NR_CHECK_ARG(n >= 0 && dim > 0 && lds >= dim && ldd >= dim, "nr_gather_rows: bad shape");
  if (n == 0) return NR_OK;
  NR_CHECK_ARG(src && dst, "nr_gather_rows: null pointer");
  NR_CHECK_DEVICE("nr_gather_rows", src, idx, dst);
  NR_DT2(dtype_in, dtype_out,
         hipLaunchKernelGGL((gather_rows_kernel<TI, TO>), dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream, n,
                            dim, (const TI*)src, lds, idx, (TO*)dst, ldd));
  NR_CHECK_LAUNCH("nr_gather_rows");
  return NR_OK;
}

extern "C" int nr_transpose(int dtype_in, int dtype_out, int64_t rows, int64_t cols, const void* src, int64_t lds,
                            void* dst, int64_t ldd, void* stream) {
  clear_error();
  NR_CHECK_ARG(NR_OKDT(dtype_in) && NR_OKDT(dtype_out), "nr_transpose: bad dtype");
  NR_CHECK_ARG(rows >= 0 && cols >= 0 && lds >= cols && ldd >= rows, "nr_transpose: bad shape");
  if (rows == 0 || cols == 0) return NR_OK;
  NR_CHECK_ARG(src && dst, "nr_transpose: null pointer");
  NR_CHECK_DEVICE("nr_transpose", src, dst);
  NR_CHECK_ARG((rows + 63) / 64 <= 65535, "nr_transpose: too many rows");
  const dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64));
  const bool b16 = dtype_in == dtype_out && dtype_in != NR_F32;
  if (b16 && rows % 8 == 0 && cols % 8 == 0 && lds % 8 == 0 && ldd % 8 == 0 && ((uintptr_t)src & 15) == 0 &&
      ((uintptr_t)dst & 15) == 0) {
    hipLaunchKernelGGL(transpose16_kernel, grid, dim3(256), 0, (hipStream_t)stream, rows, cols,
                       (const uint16_t*)src, lds, (uint16_t*)dst, ldd);
    NR_CHECK_LAUNCH("nr_transpose");
    return NR_OK;
  }
  if (dtype_in == NR_F32 && dtype_out == NR_BF16 && rows % 8 == 0 && cols % 4 == 0 && lds % 4 == 0 &&
      ldd % 8 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0) {
    hipLaunchKernelGGL(transpose_f32_bf16_kernel, grid, dim3(256), 0, (hipStream_t)stream, rows, cols,
                       (const float*)src, lds, (__bf16*)dst, ldd);
    NR_CHECK_LAUNCH("nr_transpose");
    return NR_OK;
  }
  NR_DT2(dtype_in, dtype_out,
         hipLaunchKernelGGL((transpose_kernel<TI, TO>), grid, dim3(256), 0, (hipStream_t)stream, rows, cols,
                            (const TI*)src, lds, (TO*)dst, ldd));
  NR_CHECK_LAUNCH("nr_transpose");
  return NR_OK;
}

extern "C" int nr_final_pool_fwd(int dtype, int64_t n_seg, const int64_t* off, const void* xp, int64_t ld,
                                 float* users, float* z, void* stream) {
  clear_error();
  NR_CHECK_ARG(NR_OKDT(dtype) && n_seg >= 0 && ld >= 2048, "nr_final_pool_fwd: bad args");
  if (n_seg == 0) return NR_OK;
  NR_CHECK_ARG(off && xp && users && z, "nr_final_pool_fwd: null pointer");
  NR_CHECK_DEVICE("nr_final_pool_fwd", off, xp, users, z);
  NR_CHECK_ARG(((uintptr_t)xp & 15) == 0 && ld % 4 == 0, "nr_final_pool_fwd: xp must be 16-byte aligned, ld %% 4 == 0");
  NR_DT1(dtype, hipLaunchKernelGGL((final_pool_fwd_kernel<T>), dim3((unsigned)n_seg, 4), dim3(64 * kPoolWaves), 0,
                                   (hipStream_t)stream, n_seg, off, (const T*)xp, ld, users, z));
  NR_CHECK_LAUNCH("nr_final_pool_fwd");
  return NR_OK;
}

extern "C" int nr_final_pool_bwd(int dtype, int64_t n_seg, const int64_t* off, int64_t n_rows, const void* xp,
                                 int64_t ld, const float* users, const float* z, const float* du, void* dx,
                                 int64_t lddx, void* dl, int64_t lddl, void* stream) {
  clear_error();
  NR_CHECK_ARG(NR_OKDT(dtype) && n_seg >= 0 && n_rows >= 0 && ld >= 2048 && lddx >= 1024 && lddl >= 1024,
               "nr_final_pool_bwd: bad args");
  if (n_seg == 0 && n_rows == 0) return NR_OK;
  NR_CHECK_ARG(off && xp && users && z && du && dx && dl, "nr_final_pool_bwd: null pointer");
  NR_CHECK_DEVICE("nr_final_pool_bwd", off, xp, users, z, du, dx, dl);
  NR_CHECK_ARG(((uintptr_t)xp & 15) == 0 && ((uintptr_t)dx & 15) == 0 && ((uintptr_t)dl & 15) == 0 && ld % 4 == 0 &&
                   lddx % 4 == 0 && lddl % 4 == 0,
               "nr_final_pool_bwd: xp / dx / dl must be 16-byte aligned with row strides %% 4 == 0");
  if (n_rows == 0) return NR_OK;
  NR_CHECK_ARG((n_rows + 15) / 16 <= 0x7fffffff, "nr_final_pool_bwd: too many rows");
  const unsigned grid = (unsigned)((n_rows + 15) / 16);  // 16 rows per block
  NR_DT1(dtype, hipLaunchKernelGGL((final_pool_bwd_kernel<T>), dim3(grid, 4), dim3(256), 0, (hipStream_t)stream,
                                   n_seg, off, n_rows, (const T*)xp, ld, users, z, du, (T*)dx, lddx, (T*)dl, lddl));
  NR_CHECK_LAUNCH("nr_final_pool_bwd");
  return NR_OK;
}

extern "C" int nr_cosine_margin(int64_t B, const float* users, const float* E, int64_t lde, const int32_t* pos,
                                const int32_t* neg, float margin, float* s_out, float* loss, float* du, float* dE,
                                void* stream) {
  clear_error();
  NR_CHECK_ARG(B >= 0 && lde >= 1024 && lde % 4 == 0, "nr_cosine_margin: bad args");
  if (B == 0) return NR_OK;
  NR_CHECK_ARG(users && E && pos && neg && loss && du && dE, "nr_cosine_margin: null pointer");
  NR_CHECK_DEVICE("nr_cosine_margin", users, E, pos, neg, s_out, loss, du, dE);
  hipLaunchKernelGGL(cosine_margin_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, (hipStream_t)stream, B,
                     users, E, lde, pos, neg, margin, s_out, loss, du, dE);
  NR_CHECK_LAUNCH("nr_cosine_margin");
  return NR_OK;
}

extern "C" int nr_scatter_add_rows(int dtype, int64_t n, int64_t dim, const void* src, int64_t lds,
                                   const int32_t* idx, float* dst, int64_t ldd, void* stream) {
  clear_error();
  NR_CHECK_ARG(NR_OKDT(dtype) && n >= 0 && dim > 0 && lds >= dim && ldd >= dim, "nr_scatter_add_rows: bad args");
  if (n == 0) return NR_OK;
  NR_CHECK_ARG(src && idx && dst, "nr_scatter_add_rows: null pointer");
  NR_CHECK_DEVICE("nr_scatter_add_rows", src, idx, dst);
  NR_DT1(dtype, hipLaunchKernelGGL((scatter_add_rows_kernel<T>), dim3((unsigned)n), dim3(256), 0,
                                   (hipStream_t)stream, n, dim, (const T*)src, lds, idx, dst, ldd));
  NR_CHECK_LAUNCH("nr_scatter_add_rows");
  return NR_OK;
}

extern "C" int nr_col_sum(int dtype, int64_t rows, int64_t cols, const void* src, int64_t lds, float* out,
                          void* stream) {
  clear_error();
  NR_CHECK_ARG(NR_OKDT(dtype) && rows >= 0 && cols > 0 && lds >= cols, "nr_col_sum: bad args");
  if (rows == 0) return NR_OK;
  NR_CHECK_ARG(src && out, "nr_col_sum: null pointer");
  NR_CHECK_DEVICE("nr_col_sum", src, out);
  // ~1024 blocks: column groups of 512 x row ranges (multiple of 4 rows, >= 32)
  const int64_t cgroups = (cols + 511) / 512;
  int64_t rpb = (rows * cgroups + 1023) / 1024;
  rpb = rpb < 32 ? 32 : (rpb + 3) / 4 * 4;
  NR_CHECK_ARG((rows + rpb - 1) / rpb <= 65535 && rpb <= 0x7fffffff, "nr_col_sum: too many rows");
  const dim3 grid((unsigned)cgroups, (unsigned)((rows + rpb - 1) / rpb));
  NR_DT1(dtype, hipLaunchKernelGGL((col_sum_kernel<T>), grid, dim3(256), 0, (hipStream_t)stream, rows, cols,
                                   (const T*)src, lds, (int)rpb, out));
  NR_CHECK_LAUNCH("nr_col_sum");
  return NR_OK;
}

extern "C" int nr_ln_param_grad(int dtype_in, int64_t n, int64_t dim, const void* x, int64_t ldx,
                                const int64_t* row_idx, float eps, const float* dy, int64_t lddy, float* dgamma,
                                float* dbeta, void* stream) {
  clear_error();
  NR_CHECK_ARG(dim == 1024, "nr_ln_param_grad: dim %lld unsupported", (long long)dim);
  NR_CHECK_ARG(n >= 0 && ldx >= dim && lddy >= dim, "nr_ln_param_grad: bad args");
  NR_CHECK_ARG(dtype_in == NR_F32 || dtype_in == NR_BF16 || dtype_in == NR_F16, "nr_ln_param_grad: bad dtype");
  if (n == 0) return NR_OK;
  NR_CHECK_ARG(x && dy && dgamma && dbeta, "nr_ln_param_grad: null pointer");
  NR_CHECK_DEVICE("nr_ln_param_grad", x, row_idx, dy, dgamma, dbeta);
  NR_CHECK_ARG(lddy % 4 == 0 && ((uintptr_t)dy & 15) == 0, "nr_ln_param_grad: dy rows must be 16-byte aligned");
  const int64_t g16 = (n + 15) / 16;  // ~16 rows per block: few enough blocks that the final atomics stay cheap
  const unsigned grid = (unsigned)(g16 < 256 ? g16 : 256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype_in == NR_F32)
    hipLaunchKernelGGL((ln_param_grad_kernel<float>), dim3(grid), dim3(256), 0, s, n, (const float*)x, ldx, row_idx,
                       eps, dy, lddy, dgamma, dbeta);
  else if (dtype_in == NR_BF16)
    hipLaunchKernelGGL((ln_param_grad_kernel<__bf16>), dim3(grid), dim3(256), 0, s, n, (const __bf16*)x, ldx,
                       row_idx, eps, dy, lddy, dgamma, dbeta);
  else
    hipLaunchKernelGGL((ln_param_grad_kernel<_Float16>), dim3(grid), dim3(256), 0, s, n, (const _Float16*)x, ldx,
                       row_idx, eps, dy, lddy, dgamma, dbeta);
  NR_CHECK_LAUNCH("nr_ln_param_grad");
  return NR_OK;
}

extern "C" int nr_sumsq(int64_t n, const float* x, float* out, void* stream) {
  clear_error();
  NR_CHECK_ARG(n >= 0, "nr_sumsq: bad n");
  if (n == 0) return NR_OK;
  NR_CHECK_ARG(x && out, "nr_sumsq: null pointer");
  NR_CHECK_DEVICE("nr_sumsq", x, out);
  const int64_t g = (n / 4 + 255) / 256;
  hipLaunchKernelGGL(sumsq_kernel, dim3((unsigned)(g < 1 ? 1 : g < 1024 ? g : 1024)), dim3(256), 0,
                     (hipStream_t)stream, n, x, out);
  NR_CHECK_LAUNCH("nr_sumsq");
  return NR_OK;
}

extern "C" int nr_adamw(int64_t n, float* p, const float* g, float* m, float* v, void* p_bf16, int64_t step,
                        float lr, float beta1, float beta2, float eps, float weight_decay, float max_norm,
                        const float* sumsq, void* stream) {
  clear_error();
  NR_CHECK_ARG(n >= 0 && step >= 1, "nr_adamw: bad args");
  if (n == 0) return NR_OK;
  NR_CHECK_ARG(p && g && m && v, "nr_adamw: null pointer");
  NR_CHECK_DEVICE("nr_adamw", p, g, m, v, p_bf16, sumsq);
  const float bc1 = (float)(1.0 - pow((double)beta1, (double)step));
  const float bc2s = (float)sqrt(1.0 - pow((double)beta2, (double)step));
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v,
                     (__bf16*)p_bf16, lr, beta1, beta2, eps, weight_decay, bc1, bc2s, max_norm, sumsq);
  NR_CHECK_LAUNCH("nr_adamw");
  return NR_OK;
}

extern "C" int nr_splitk_fixup(int dtype_out, int epilogue, int64_t rows, int64_t N, int parts, const float* partials,
                               const float* bias, const void* R, int64_t ldr, void* C, int64_t ldc, int64_t row0,
                               uint64_t seed, float p, float scale, void* stream) {
  clear_error();
  NR_CHECK_ARG(NR_OKDT(dtype_out) && rows >= 0 && N > 0 && N % 4 == 0 && parts >= 1 && ldc >= N && row0 >= 0,
               "nr_splitk_fixup: bad args");
  NR_CHECK_ARG(epilogue == NR_EPI_NONE || epilogue == NR_EPI_RELU_DROPOUT || epilogue == NR_EPI_DRELU ||
                   epilogue == NR_EPI_RESADD || epilogue == NR_EPI_EXP,
               "nr_splitk_fixup: epilogue %d unsupported", epilogue);
  NR_CHECK_ARG(p >= 0.f && p < 1.f, "nr_splitk_fixup: dropout p outside [0, 1)");
  if (rows == 0) return NR_OK;
  NR_CHECK_ARG(partials && C && ((epilogue != NR_EPI_DRELU && epilogue != NR_EPI_RESADD) || (R && ldr >= N)),
               "nr_splitk_fixup: null pointer");
  NR_CHECK_ARG(((uintptr_t)partials & 15) == 0, "nr_splitk_fixup: partials must be 16-byte aligned");
  NR_CHECK_DEVICE("nr_splitk_fixup", partials, bias, R, C);
  // dropout threshold and scale exactly as nr_gemm_relu_dropout forms them
  const uint32_t thr = dropout_threshold(p);
  if (epilogue == NR_EPI_RELU_DROPOUT) scale = 1.0f / (1.0f - p);
  const int64_t quads = rows * (N / 4);
  NR_CHECK_ARG((quads + 255) / 256 <= 0x7fffffff, "nr_splitk_fixup: too many rows");
  const dim3 grid((unsigned)((quads + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
#define NR_FIX(E)                                                                                                   \
  NR_DT1(dtype_out, hipLaunchKernelGGL((splitk_fixup_kernel<E, T>), grid, dim3(256), 0, s, rows, N, parts, partials, \
                                       bias, (const T*)R, ldr, (T*)C, ldc, row0, seed, thr, scale))
  if (epilogue == NR_EPI_RELU_DROPOUT) NR_FIX(NR_EPI_RELU_DROPOUT);
  else if (epilogue == NR_EPI_DRELU) NR_FIX(NR_EPI_DRELU);
  else if (epilogue == NR_EPI_RESADD) NR_FIX(NR_EPI_RESADD);
  else if (epilogue == NR_EPI_EXP) NR_FIX(NR_EPI_EXP);
  else NR_FIX(NR_EPI_NONE);
#undef NR_FIX
  NR_CHECK_LAUNCH("nr_splitk_fixup");
  return NR_OK;
}

static unsigned rowwave_grid(int64_t units) {  // 4 waves (units) per block, <= 2048 blocks, grid-strided
  const int64_t b = (units + 3) / 4;
  return (unsigned)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

extern "C" int nr_layernorm_bwd(int64_t n, int64_t dim, const float* x, int64_t ldx, const float* gamma, float eps,
                                const float* dy, int64_t lddy, const float* dres, int64_t ldr, float* dx,
                                int64_t lddx, void* stream) {
  clear_error();
  NR_CHECK_ARG(dim == 1024, "nr_layernorm_bwd: dim %lld unsupported", (long long)dim);
  NR_CHECK_ARG(n >= 0 && ldx >= dim && lddy >= dim && lddx >= dim && (!dres || ldr >= dim), "nr_layernorm_bwd: bad args");
  if (n == 0) return NR_OK;
  NR_CHECK_ARG(x && dy && dx, "nr_layernorm_bwd: null pointer");
  NR_CHECK_DEVICE("nr_layernorm_bwd", x, gamma, dy, dres, dx);
  NR_CHECK_ARG(ldx % 4 == 0 && lddy % 4 == 0 && lddx % 4 == 0 && (!dres || ldr % 4 == 0) &&
                   (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx | (uintptr_t)dres | (uintptr_t)gamma) & 15) == 0,
               "nr_layernorm_bwd: rows must be 16-byte aligned");
  hipLaunchKernelGGL(layernorm_bwd_kernel, dim3(rowwave_grid(n)), dim3(256), 0, (hipStream_t)stream, n, x, ldx, gamma,
                     eps, dy, lddy, dres, ldr, dx, lddx);
  NR_CHECK_LAUNCH("nr_layernorm_bwd");
  return NR_OK;
}

extern "C" int nr_softmax64_bwd(int dtype_out, int64_t rows, int64_t cols, const float* p, int64_t ldp, const float* dp,
                                int64_t lddp, void* ds, int64_t ldds, void* stream) {
  clear_error();
  NR_CHECK_ARG(dtype_out == NR_F32 || dtype_out == NR_BF16, "nr_softmax64_bwd: dtype_out must be f32 or bf16");
  NR_CHECK_ARG(rows >= 0 && cols > 0 && cols % 64 == 0 && ldp >= cols && lddp >= cols && ldds >= cols,
               "nr_softmax64_bwd: bad args (cols must be a multiple of 64)");
  if (rows == 0) return NR_OK;
  NR_CHECK_ARG(p && dp && ds, "nr_softmax64_bwd: null pointer");
  NR_CHECK_DEVICE("nr_softmax64_bwd", p, dp, ds);
  const int64_t gpr = cols / 64, ng = rows * gpr;
  if (dtype_out == NR_F32)
    hipLaunchKernelGGL((softmax64_bwd_kernel<float>), dim3(rowwave_grid(ng)), dim3(256), 0, (hipStream_t)stream, ng,
                       gpr, p, ldp, dp, lddp, (float*)ds, ldds);
  else
    hipLaunchKernelGGL((softmax64_bwd_kernel<__bf16>), dim3(rowwave_grid(ng)), dim3(256), 0, (hipStream_t)stream, ng,
                       gpr, p, ldp, dp, lddp, (__bf16*)ds, ldds);
  NR_CHECK_LAUNCH("nr_softmax64_bwd");
  return NR_OK;
}

static unsigned elem4_grid(int64_t total) {
  const int64_t b = (total / 4 + 255) / 256;
  return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

extern "C" int nr_geglu_fwd(int dtype_out, int64_t rows, int64_t f, const float* g, int64_t ldg, void* z, int64_t ldz,
                            void* stream) {
  clear_error();
  NR_CHECK_ARG(dtype_out == NR_F32 || dtype_out == NR_BF16, "nr_geglu_fwd: dtype_out must be f32 or bf16");
  NR_CHECK_ARG(rows >= 0 && f > 0 && f % 4 == 0 && ldg >= 2 * f && ldz >= f && ldg % 4 == 0 && ldz % 4 == 0,
               "nr_geglu_fwd: bad args");
  if (rows == 0) return NR_OK;
  NR_CHECK_ARG(g && z, "nr_geglu_fwd: null pointer");
  NR_CHECK_DEVICE("nr_geglu_fwd", g, z);
  NR_CHECK_ARG((((uintptr_t)g | (uintptr_t)z) & 15) == 0, "nr_geglu_fwd: 16-byte alignment required");
  if (dtype_out == NR_F32)
    hipLaunchKernelGGL((geglu_fwd_kernel<float>), dim3(elem4_grid(rows * f)), dim3(256), 0, (hipStream_t)stream, rows,
                       f, g, ldg, (float*)z, ldz);
  else
    hipLaunchKernelGGL((geglu_fwd_kernel<__bf16>), dim3(elem4_grid(rows * f)), dim3(256), 0, (hipStream_t)stream, rows,
                       f, g, ldg, (__bf16*)z, ldz);
  NR_CHECK_LAUNCH("nr_geglu_fwd");
  return NR_OK;
}

extern "C" int nr_geglu_bwd(int dtype_out, int64_t rows, int64_t f, const float* g, int64_t ldg, const float* dz,
                            int64_t lddz, void* dg, int64_t lddg, void* stream) {
  clear_error();
  NR_CHECK_ARG(dtype_out == NR_F32 || dtype_out == NR_BF16, "nr_geglu_bwd: dtype_out must be f32 or bf16");
  NR_CHECK_ARG(rows >= 0 && f > 0 && f % 4 == 0 && ldg >= 2 * f && lddz >= f && lddg >= 2 * f && ldg % 4 == 0 &&
                   lddz % 4 == 0 && lddg % 4 == 0,
               "nr_geglu_bwd: bad args");
  if (rows == 0) return NR_OK;
  NR_CHECK_ARG(g && dz && dg, "nr_geglu_bwd: null pointer");
  NR_CHECK_DEVICE("nr_geglu_bwd", g, dz, dg);
  NR_CHECK_ARG((((uintptr_t)g | (uintptr_t)dz | (uintptr_t)dg) & 15) == 0, "nr_geglu_bwd: 16-byte alignment required");
  if (dtype_out == NR_F32)
    hipLaunchKernelGGL((geglu_bwd_kernel<float>), dim3(elem4_grid(rows * f)), dim3(256), 0, (hipStream_t)stream, rows,
                       f, g, ldg, dz, lddz, (float*)dg, lddg);
  else
    hipLaunchKernelGGL((geglu_bwd_kernel<__bf16>), dim3(elem4_grid(rows * f)), dim3(256), 0, (hipStream_t)stream, rows,
                       f, g, ldg, dz, lddz, (__bf16*)dg, lddg);
  NR_CHECK_LAUNCH("nr_geglu_bwd");
  return NR_OK;
}
