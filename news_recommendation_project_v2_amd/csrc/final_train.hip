// Config-5 training step with the FinalAttention pooler -- the pairing the
// reference's scripts/train_v3.py trains (AttentionAttentionTrainer,
// trainer.py:1030-1117; FinalAttention.forward, modeling_utils.py:195-228) --
// forward and backward of one batch as one C call (nr_final_train_step,
// include/newsrec.h):
//
//   E  = g_mlp_LN(last token)                               token model (attention.py:193)
//   per history slot (packed valid rows, CSR order, zero rows up to Hp = pad64(Hs)):
//        S = E[hist];  X1 = drop(relu(S W1^T + b1));  X2 = drop(relu(X1 W2^T + b2))
//        X = X2 W3^T + b3;  Y = drop(relu(X W4^T + b4));  P = exp(Y W5^T)
//   per batch row: u_d = sum_i X_id P_id / (sum_i P_id + 1e-10)   (modeling_utils.py:224-228)
//        loss = MarginRankingLoss(2)(cos(u, E[pos]), cos(u, E[neg]))   (trainer.py:1058-1066)
//   backward: pool' -> dL (logits of linear5), dXp (X) -> dY = drop'(dL W5) -> dX = dY W4 + dXp
//        -> dZ2 = drop'(dX W3) -> dZ1 = drop'(dZ2 W2)
//        weight grads dW5 = dL^T Y, dW4 = dY^T X, dW3 = dX^T X2, dW2 = dZ2^T X1, dW1 = dZ1^T S
//        bias grads = column sums of dY, dX, dZ2, dZ1; token LayerNorm parameter grads.
//   The history gather's gradient dS = dZ1 W1 is never formed: its only consumer is
//   the token LayerNorm's parameters (E is the LN of the last token), and with
//   S = xhat gamma + beta its contributions are sum_slots dS = g_b1 W1 and
//   sum_slots dS o xhat = sum_h W1[h] o M[h], M = dZ1^T xhat -- the weight-grad GEMM
//   of W1 run on xhat instead of S, dW1 = gamma o M + g_b1 (x) beta (w1_fold_kernel):
//   the dS GEMM (70 GFLOP), its scatter into the U rows and their LN reduction go.
//
// FinalAttention runs once per VALID history slot (the reference's padded slots
// carry zero pooling weight and so zero gradient).  Dropout: the counter-hash
// stream of nr_gemm_relu_dropout (oracle/train_ref.py restates it).
//
// bf16 (the throughput mode): every GEMM on the persistent MFMA kernel, the
// N = 4096 ones with the rows past the last whole tile round as split-K slices
// (+ nr_splitk_fixup); the bias gradients as f32 column sums written by the
// data-grad GEMMs' epilogues (no re-read of dY / dX / dZ2 / dZ1); the five
// weight-grad GEMMs as ONE grouped TN launch that reads the row-major
// activations through transposed LDS reads (no transposed copies); the five
// weight transposes the data-grad GEMMs need on a side stream beside the
// forward's first N = 1024 GEMM.  The token LN (E) is never stored as a [U][D]
// table: the slot kernel computes it per history slot from the token states,
// the cosine kernel per pos / neg row.  f32 (the parity mode): the same sequence
// on the exact-f32 MFMA tile kernels, with explicit transposes for the weight
// grads.
#include "nr_common.h"

namespace nr {
namespace ft {

constexpr int64_t D = 1024, H = 4096;
// K-slices of a split-K tail: K = 4096 as 8 (26.7 vs 33.1 us as 4; tools/tail_probe.py,
// profiles/round5/train/tail_probe_r5m.jsonl).  Only the K = 4096 GEMMs split their
// tail rows (split_tail below); the K = 1024 ones take the persistent kernel's half tile.
constexpr int kSplit = 8;
// sum-of-squares partials of the bf16 step: 512 weight-grad tiles, then the W1 fold's
// 16 x 64 blocks, the bias reduction's 208 blocks, the token LN reduction's 16
constexpr int kSqTn = 512, kSqFold = (1024 / 64) * (4096 / 64), kSqBias = (3 * 4096 + 1024) / 64, kSqLn = 1024 / 64;
constexpr int kSqParts = kSqTn + kSqFold + kSqBias + kSqLn;

static int64_t pad64(int64_t n) { return n < 64 ? 64 : (n + 63) / 64 * 64; }
static int64_t al(int64_t b) { return (b + 255) / 256 * 256; }

// ------------------------------------------------------------------ small kernels
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
template <typename T>
__device__ __forceinline__ void st4(T* p, const float v[4]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
  } else {
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<b4*>(p) = __builtin_convertvector(f4{v[0], v[1], v[2], v[3]}, b4);
  }
}

// The token model's output row of news n (g_mlp_layernorm without its affine, eps
// 1e-12: the arithmetic of gather_ln_kernel, rowops.hip, so the bits are those of
// nr_gather_layernorm): lane's 4 x 4 columns 256 j + 4 lane .. +3 of xhat.  TT =
// the token states' type (f32 / bf16 / f16).
template <typename TT>
__device__ __forceinline__ void tok_xhat(const TT* row, int lane, float (&v)[4][4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const TT* p = row + j * 256 + lane * 4;
    if constexpr (sizeof(TT) == 4) {
      ld4<float>((const float*)p, v[j]);
    } else if constexpr (std::is_same<TT, _Float16>::value) {
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      const h4 h = *reinterpret_cast<const h4*>(p);
      v[j][0] = (float)h[0]; v[j][1] = (float)h[1]; v[j][2] = (float)h[2]; v[j][3] = (float)h[3];
    } else {
      ld4<__bf16>((const __bf16*)p, v[j]);
    }
  }
  float sm = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) sm += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
  const float mean = wave_sum(sm) / (float)D;
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

struct ZList {  // zero up to 8 f32 ranges in one launch
  float* p[8];
  int64_t len[8];
  int n;
};
__global__ __launch_bounds__(256) void zero_kernel(ZList z) {
  for (int i = 0; i < z.n; ++i)
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < z.len[i]; j += (int64_t)gridDim.x * 256)
      z.p[i][j] = 0.f;
}

// Slot rows i < Hp: xhat = the token LN (no affine) of the last token of news
// hist[i], computed here per slot from the token states (no [U][D] LN table:
// Hs ~ U at the benchmark batch, and the token rows are half the bytes),
// S[i] = xhat gamma + beta and XH[i] = xhat (TA; zero rows past Hs).  The pos / neg
// rows' LN is formed by cos_pairs_kernel.  One wave per row, 4 columns per lane.
template <typename TA, typename TT>
__global__ __launch_bounds__(256) void slots_kernel(int64_t Hp, int64_t Hs, const TT* __restrict__ tok,
                                                    const int32_t* __restrict__ hist, const float* __restrict__ g,
                                                    const float* __restrict__ b, TA* __restrict__ S,
                                                    TA* __restrict__ XH) {
  const int lane = threadIdx.x & 63;
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < Hp; i += (int64_t)gridDim.x * 4) {
    const int64_t r = i < Hs ? (int64_t)hist[i] : -1;  // wave-uniform
    float v[4][4] = {};
    if (r >= 0) tok_xhat<TT>(tok + r * D, lane, v);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t c = 256 * j + 4 * lane;
      float gg[4], bb[4], e[4];
      ld4<float>(g + c, gg);
      ld4<float>(b + c, bb);
#pragma unroll
      for (int t = 0; t < 4; ++t) e[t] = r >= 0 ? fmaf(v[j][t], gg[t], bb[t]) : 0.f;
      st4<TA>(S + i * D + c, e);
      st4<TA>(XH + i * D + c, v[j]);
    }
  }
}

// The token LayerNorm's part of the backward without the dS GEMM.  The history
// gather's gradient dS = dZ1 W1 only ever reaches the token LN parameters (E is
// the last-token LN, attention.py:193), and with S = xhat gamma + beta:
//   sum_slots dS = g_b1 W1                         -> dbeta  += g_b1 W1
//   sum_slots dS o xhat = sum_h W1[h] o M[h]       -> dgamma += sum_h W1[h] o M[h],  M = dZ1^T XH
//   dW1 = dZ1^T S = gamma o M + g_b1 (x) beta      (M computed in dW1's buffer, rewritten here)
// Block = 64 columns x 64 rows h (4 groups of 16 rows, folded in LDS); per-chunk
// partials [H / 64][2][D] summed in chunk order by ln_reduce_kernel (deterministic).
// (block (bx, by) of nbx x H / 64; gb1p[h - hbase] = g_b1[h] for the block's 64 rows h)
template <typename TA>
__device__ __forceinline__ void w1_fold_body(int bx, int by, int nbx, const TA* __restrict__ W1, float* __restrict__ gW1,
                                             const float* gb1p, int64_t hbase, const float* __restrict__ g,
                                             const float* __restrict__ b, float* __restrict__ part,
                                             float* __restrict__ sqp) {
  __shared__ float red[2][4][64];
  __shared__ float rsq[4];
  const int grp = threadIdx.x >> 6, cl = threadIdx.x & 63;
  const int64_t c = (int64_t)bx * 64 + cl;
  const int64_t h0 = (int64_t)by * 64 + grp * 16;
  const float gc = g[c], bc = b[c];
  float sg = 0.f, sb = 0.f, sq = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int64_t h = h0 + k;
    const float w = (float)W1[h * D + c], m = gW1[h * D + c], gh = gb1p[h - hbase];
    sg = fmaf(w, m, sg);
    sb = fmaf(w, gh, sb);
    const float dw = fmaf(gc, m, bc * gh);
    gW1[h * D + c] = dw;
    sq = fmaf(dw, dw, sq);
  }
  red[0][grp][cl] = sg;
  red[1][grp][cl] = sb;
  if (sqp) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) sq += __shfl_xor(sq, o, 64);
    if (cl == 0) rsq[grp] = sq;
  }
  __syncthreads();
  if (sqp && threadIdx.x == 0) sqp[(int64_t)by * nbx + bx] = (rsq[0] + rsq[1]) + (rsq[2] + rsq[3]);
  if (threadIdx.x < 128) {
    const int w = threadIdx.x >> 6;
    const float v = (red[w][0][cl] + red[w][1][cl]) + (red[w][2][cl] + red[w][3][cl]);
    part[(int64_t)by * 2 * D + w * D + c] = v;
  }
}
// f32 mode: g_b1 already summed (nr_col_sum)
template <typename TA>
__global__ __launch_bounds__(256) void w1_fold_kernel(const TA* __restrict__ W1, float* __restrict__ gW1,
                                                      const float* __restrict__ gb1, const float* __restrict__ g,
                                                      const float* __restrict__ b, float* __restrict__ part,
                                                      float* __restrict__ sqp) {
  w1_fold_body<TA>((int)blockIdx.x, (int)blockIdx.y, (int)gridDim.x, W1, gW1, gb1, 0, g, b, part, sqp);
}
// dg[c] = sum_k part[k][0][c], db[c] = sum_k part[k][1][c] over the W1 fold's and the
// pairs' chunks: 64 columns x 4 chunk groups per block (with sqp: their sum of squares)
__global__ __launch_bounds__(256) void ln_reduce_kernel(int nchunk, const float* __restrict__ part,
                                                        float* __restrict__ dg, float* __restrict__ db,
                                                        float* __restrict__ sqp) {
  __shared__ float red[2][4][64];
  const int grp = threadIdx.x >> 6, cl = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 64 + cl;
  float sg = 0.f, sb = 0.f;
  for (int k = grp; k < nchunk; k += 4) {
    sg += part[(int64_t)k * 2 * D + c];
    sb += part[(int64_t)k * 2 * D + D + c];
  }
  red[0][grp][cl] = sg;
  red[1][grp][cl] = sb;
  __syncthreads();
  if (threadIdx.x < 64) {
    const float vg = (red[0][0][cl] + red[0][1][cl]) + (red[0][2][cl] + red[0][3][cl]);
    const float vb = (red[1][0][cl] + red[1][1][cl]) + (red[1][2][cl] + red[1][3][cl]);
    dg[c] = vg;
    db[c] = vb;
    if (sqp) {
      float q = fmaf(vg, vg, vb * vb);
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) q += __shfl_xor(q, o, 64);
      if (cl == 0) sqp[blockIdx.x] = q;
    }
  }
}
// *out = sum of the n grad-norm partials (the step's grad norm^2: clip_grad_norm_
// reads it, trainer.py:1067-1070).  One block, fixed order.
__global__ __launch_bounds__(256) void sq_total_kernel(int64_t n, const float* __restrict__ part,
                                                       float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += part[i];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = (red[0] + red[1]) + (red[2] + red[3]);
}

// F.cosine_similarity(u, E[pos / neg]) with the per-vector 1e-8 clamp and
// MarginRankingLoss(margin) (trainer.py:1058-1066), as nr_cosine_margin, but the
// gradients of E[pos[b]] / E[neg[b]] are written per pair ([2B][D]: no atomics
// into a [U][D] dE) and the per-row loss terms kept for an ordered sum: E is
// the token LN's output, so those rows only feed pair_ln_kernel.  One wave per row.
template <typename TT>
__global__ __launch_bounds__(256) void cos_pairs_kernel(int64_t B, const float* __restrict__ users,
                                                        const TT* __restrict__ tok, float* __restrict__ xpair,
                                                        const float* __restrict__ tg,
                                                        const float* __restrict__ tb, const int32_t* __restrict__ pos,
                                                        const int32_t* __restrict__ neg, float margin,
                                                        float* __restrict__ lrow, float* __restrict__ du,
                                                        float* __restrict__ gpair) {
  constexpr float EPS = 1e-8f;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float u[4][4], ep[4][4], en[4][4];
  float uu = 0.f, pp = 0.f, nn = 0.f, up = 0.f, un = 0.f;
  // E[n] = xhat[n] gamma + beta (the token LN's output), as slots_kernel forms S;
  // the pairs' xhat rows kept for pair_ln_kernel (xpair [2B][D]: pos rows, then neg)
  tok_xhat<TT>(tok + (int64_t)pos[b] * D, lane, ep);
  tok_xhat<TT>(tok + (int64_t)neg[b] * D, lane, en);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = j * 256 + lane * 4;
    float gg[4], bb[4];
    st4<float>(xpair + b * D + e, ep[j]);
    st4<float>(xpair + (B + b) * D + e, en[j]);
    ld4<float>(users + b * D + e, u[j]);
    ld4<float>(tg + e, gg);
    ld4<float>(tb + e, bb);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      ep[j][t] = fmaf(ep[j][t], gg[t], bb[t]);
      en[j][t] = fmaf(en[j][t], gg[t], bb[t]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      uu = fmaf(u[j][t], u[j][t], uu);
      pp = fmaf(ep[j][t], ep[j][t], pp);
      nn = fmaf(en[j][t], en[j][t], nn);
      up = fmaf(u[j][t], ep[j][t], up);
      un = fmaf(u[j][t], en[j][t], un);
    }
  }
  auto wsum = [](float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  };
  uu = wsum(uu); pp = wsum(pp); nn = wsum(nn); up = wsum(up); un = wsum(un);
  const float nu = sqrtf(uu), np_ = sqrtf(pp), nq = sqrtf(nn);
  const float iu = 1.0f / fmaxf(nu, EPS), ip = 1.0f / fmaxf(np_, EPS), iq = 1.0f / fmaxf(nq, EPS);
  const float sp = up * iu * ip, sn = un * iu * iq;
  const float v = margin - (sp - sn);
  const float act = v >= 0.f ? 1.0f : 0.0f;  // clamp_min backward passes where input >= min
  const float gsp = -act / (float)B, gsn = act / (float)B;
  if (lane == 0) lrow[b] = fmaxf(v, 0.f) / (float)B;
  const float cu = nu > EPS ? 1.f : 0.f, cp = np_ > EPS ? 1.f : 0.f, cq = nq > EPS ? 1.f : 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = j * 256 + lane * 4;
    float g[4], gp[4], gn[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float uh = u[j][t] * iu, ph = ep[j][t] * ip, qh = en[j][t] * iq;
      g[t] = gsp * (ph - cu * sp * uh) * iu + gsn * (qh - cu * sn * uh) * iu;
      gp[t] = gsp * (uh - cp * sp * ph) * ip;
      gn[t] = gsn * (uh - cq * sn * qh) * iq;
    }
    st4<float>(du + b * D + e, g);
    st4<float>(gpair + b * D + e, gp);
    st4<float>(gpair + (B + b) * D + e, gn);
  }
}

// The pairs' part of the token LN parameter grads: chunk k of the 2B pair rows
// (rows k, k + kPairChunks, ...) -> partials part[k][0][c] = sum g o xhat,
// part[k][1][c] = sum g, in the layout of the W1 fold's chunk partials (placed
// after them, ln_reduce_kernel sums both).  Block = 64 columns x 4 row groups;
// grid (D / 64, kPairChunks).  Block (0, 0)'s first wave also writes the loss as
// the ordered (fixed tree) sum of the per-row terms.
constexpr int kPairChunks = 8;
__global__ __launch_bounds__(256) void pair_ln_kernel(int64_t B, const float* __restrict__ gpair,
                                                      const float* __restrict__ xpair, const float* __restrict__ lrow,
                                                      float* __restrict__ part, float* __restrict__ loss) {
  __shared__ float red[2][4][64];
  const int grp = threadIdx.x >> 6, cl = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 64 + cl;
  const int64_t step = (int64_t)kPairChunks * 4;
  float sg = 0.f, sb = 0.f;
#pragma unroll 4
  for (int64_t r = (int64_t)blockIdx.y + kPairChunks * grp; r < 2 * B; r += step) {
    const float gv = gpair[r * D + c];
    sg = fmaf(gv, xpair[r * D + c], sg);
    sb += gv;
  }
  red[0][grp][cl] = sg;
  red[1][grp][cl] = sb;
  __syncthreads();
  if (threadIdx.x < 64) {
    part[(int64_t)blockIdx.y * 2 * D + c] = (red[0][0][cl] + red[0][1][cl]) + (red[0][2][cl] + red[0][3][cl]);
    part[(int64_t)blockIdx.y * 2 * D + D + c] = (red[1][0][cl] + red[1][1][cl]) + (red[1][2][cl] + red[1][3][cl]);
    if (blockIdx.x == 0 && blockIdx.y == 0) {
      float l = 0.f;
      for (int64_t r = threadIdx.x; r < B; r += 64) l += lrow[r];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) l += __shfl_xor(l, o, 64);
      if (threadIdx.x == 0) *loss = l;
    }
  }
}

// A DRELU split-K tail in one launch: C = drop'(sum_s P[s] + 0) against the forward
// output R, as nr_splitk_fixup's DRELU (the same f32 sum order and rounding), and
// the stored values' column sums per 32-row block into CS row cs_row0 + block (the
// tail's rows of the CS layout, after the persistent GEMM's 128-row ones), folded
// in LDS in a fixed order.  Block = 64 columns (8 lanes x 8) x 32 rows, one row
// per thread: 256 blocks for a 128-row tail of N = 4096.
template <typename TA>
__global__ __launch_bounds__(256) void fixup_drelu_cs_kernel(int64_t cs_row0, int64_t rows, int64_t N, int parts,
                                                             const float* __restrict__ P, const TA* __restrict__ R,
                                                             int64_t ldr, TA* __restrict__ C, int64_t ldc, float scale,
                                                             float* __restrict__ cs) {
  __shared__ float red[32][64];
  const int rg = threadIdx.x >> 3, cl = threadIdx.x & 7;
  const int64_t c = (int64_t)blockIdx.x * 64 + 8 * cl;
  const int64_t r = (int64_t)blockIdx.y * 32 + rg;
  float y[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (r < rows) {
    float v[8], w[8], rv[8];
    ld4<float>(P + r * N + c, v);
    ld4<float>(P + r * N + c + 4, v + 4);
    for (int s = 1; s < parts; ++s) {
      ld4<float>(P + ((int64_t)s * rows + r) * N + c, w);
      ld4<float>(P + ((int64_t)s * rows + r) * N + c + 4, w + 4);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += w[k];
    }
    ld4<TA>(R + r * ldr + c, rv);
    ld4<TA>(R + r * ldr + c + 4, rv + 4);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float x = v[k] + 0.f;  // (no bias: as the fixup's x + 0)
      y[k] = rv[k] > 0.f ? x * scale : 0.f;
    }
    st4<TA>(C + r * ldc + c, y);
    st4<TA>(C + r * ldc + c + 4, y + 4);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rg][8 * cl + k] = y[k];  // pre-rounding, as the persistent GEMM's CS epilogue
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) t += red[k][threadIdx.x];
    cs[(cs_row0 + blockIdx.y) * N + (int64_t)blockIdx.x * 64 + threadIdx.x] = t;
  }
}

// g[c] = sum_r part[r][c] over up to 4 (partials, rows, cols, out) problems: the
// bias gradients.  Block = 64 columns (16 lanes x 4, 16-B loads) x 16 row groups,
// folded in LDS in a fixed order (deterministic).
struct RSum {
  const float* part[4];
  float* out[4];
  int64_t rows[4], cols[4];
  int n;
};
__device__ __forceinline__ void rowsum_body(const RSum& r, int bid, float* __restrict__ sqp) {
  __shared__ float red[16][64];
  int64_t c0 = (int64_t)bid * 64;
  int i = 0;
  while (i < r.n && c0 >= r.cols[i]) c0 -= r.cols[i++];
  if (i >= r.n) {  // block-uniform
    if (sqp && threadIdx.x == 0) sqp[bid] = 0.f;
    return;
  }
  const int grp = threadIdx.x >> 4, q = threadIdx.x & 15;
  const float* p = r.part[i];
  const int64_t cols = r.cols[i];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t k = grp; k < r.rows[i]; k += 16) {
    float v[4];
    ld4<float>(p + k * cols + c0 + 4 * q, v);
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] += v[t];
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) red[grp][4 * q + t] = acc[t];
  __syncthreads();
  if (threadIdx.x < 64) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][threadIdx.x];
    r.out[i][c0 + threadIdx.x] = s;
    if (sqp) {
      float q = s * s;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) q += __shfl_xor(q, o, 64);
      if (threadIdx.x == 0) sqp[bid] = q;
    }
  }
}

// bf16: the bias grads (rowsum blocks 0 .. nrs - 1) and the W1 fold (the rest, D / 64 x
// H / 64 blocks) as one launch.  A fold block needs g_b1 over its 64 rows h: it sums
// them from cs1 itself with rowsum_body's arithmetic for b1's block h / 64 (the same
// bits as the g_b1 it writes).
template <typename TA>
__global__ __launch_bounds__(256) void bias_fold_kernel(RSum r, int nrs, float* __restrict__ sq_rs, const TA* __restrict__ W1,
                                                        float* __restrict__ gW1, const float* __restrict__ g,
                                                        const float* __restrict__ b, float* __restrict__ part,
                                                        float* __restrict__ sq_fold) {
  __shared__ float gb1s[64];
  const int id = (int)blockIdx.x;
  if (id < nrs) {  // block-uniform
    rowsum_body(r, id, sq_rs);
    return;
  }
  const int f = id - nrs, nbx = (int)(D / 64), bx = f % nbx, by = f / nbx;
  {
    __shared__ float red[16][64];
    const int grp = threadIdx.x >> 4, q = threadIdx.x & 15;
    const int64_t c0 = (int64_t)by * 64;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int64_t k = grp; k < r.rows[0]; k += 16) {
      float v[4];
      ld4<float>(r.part[0] + k * r.cols[0] + c0 + 4 * q, v);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] += v[t];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) red[grp][4 * q + t] = acc[t];
    __syncthreads();
    if (threadIdx.x < 64) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) s += red[k][threadIdx.x];
      gb1s[threadIdx.x] = s;
    }
    __syncthreads();
  }
  w1_fold_body<TA>(bx, by, nbx, W1, gW1, gb1s, (int64_t)by * 64, g, b, part, sq_fold);
}

// ------------------------------------------------------------------ workspace
struct Layout {
  int64_t Hp, es, mm, csr, csr3;
  int64_t xpair, S, XH, X1, X2, XP, Y, users, z, du, gpair, lrow, dXp, dL, dY, dX, dZ2, dZ1, w1p, sqp;
  int64_t W2t, W3t, W4t, W5t, skP, cs4, cs3, cs2, cs1;
  int64_t T[10];  // f32 mode: the weight-grad operands transposed
  int64_t total;
};

// Rows of the K = 4096, N = 4096 GEMMs that fill whole rounds of 256x256 tiles
// over the CUs (the rest run as kSplit K-slices + fixup); Hp when no split pays.
// The K = 1024 ones run all Hp rows on the persistent kernel, whose half-tile
// tail (the last partial round cut into 128-row units) costs half a 16-step
// tile there, less than the split tail's two launches (tools/halves_probe.py:
// 71.9 vs 59.0 + 19.0 us at Hp = 8,320; in the step 1.735-1.739 -> 1.710-1.719
// ms, profiles/round6/final_unsplit); at K = 4096 half a tile is 64 steps and
// the K-slices win (27 vs 46 us).
static constexpr bool split_tail(int64_t K) { return K > 1024; }
static int64_t main_rows(int dtype, int64_t Hp, int ncu) {
  const int64_t ntn = H / 256;
  if (dtype != NR_BF16 || Hp % 256 == 0 || ncu % ntn) return Hp;
  const int64_t per = 256 * (ncu / ntn);
  const int64_t mm = Hp / per * per;
  const int64_t tail_tiles = (Hp - mm + 255) / 256 * ntn;
  return mm > 0 && tail_tiles * 4 <= ncu ? mm : Hp;
}

static Layout layout(int dtype, int64_t B, int64_t U, int64_t Hs, int ncu) {
  Layout L{};
  L.Hp = pad64(Hs);
  L.es = dtype == NR_F32 ? 4 : 2;
  L.mm = main_rows(dtype, L.Hp, ncu);
  // CS partial rows (bf16 column-sum epilogues): 128-row blocks of the persistent
  // GEMM over rows [0, mm), then 32-row blocks of a split-K tail (fixup_drelu_cs_kernel);
  // csr3 (128-row blocks over all Hp rows, never more than csr) for the GEMMs
  // with no tail split (dX, N = 1024; dY and dZ2, K = 1024)
  L.csr3 = (L.Hp + 127) / 128;
  L.csr = L.mm < L.Hp ? L.mm / 128 + (L.Hp - L.mm + 31) / 32 : L.csr3;
  const int64_t Hp = L.Hp, es = L.es, Bp = pad64(B);
  int64_t o = 0;
  auto take = [&](int64_t bytes) { const int64_t r = o; o += al(bytes); return r; };
  L.xpair = take(2 * B * D * 4);
  L.S = take(Hp * D * es); L.XH = take(Hp * D * es); L.X1 = take(Hp * H * es); L.X2 = take(Hp * H * es); L.XP = take(Hp * 2 * D * es);
  L.Y = take(Hp * H * es);
  L.users = take(Bp * D * 4); L.z = take(Bp * D * 4); L.du = take(Bp * D * 4); L.gpair = take(2 * B * D * 4);
  L.lrow = take(Bp * 4);
  L.sqp = take(kSqParts * 4);
  L.dXp = take(Hp * D * es); L.dL = take(Hp * D * es); L.dY = take(Hp * H * es); L.dX = take(Hp * D * es);
  L.dZ2 = take(Hp * H * es); L.dZ1 = take(Hp * H * es); L.w1p = take((H / 64 + kPairChunks) * 2 * D * 4);
  L.W2t = take(H * H * es); L.W3t = take(H * D * es); L.W4t = take(D * H * es);
  L.W5t = take(H * D * es);
  if (dtype == NR_BF16) {
    L.skP = take((int64_t)kSplit * (Hp - L.mm) * H * 4);
    L.cs4 = take(L.csr * H * 4); L.cs3 = take(L.csr3 * D * 4); L.cs2 = take(L.csr * H * 4); L.cs1 = take(L.csr * H * 4);
  } else {
    // dL^T, Y^T, dY^T, X^T, dX^T, X2^T, dZ2^T, X1^T, dZ1^T, XH^T
    const int64_t w[10] = {D, H, H, D, D, H, H, H, H, D};
    for (int i = 0; i < 10; ++i) L.T[i] = take(w[i] * Hp * es);
  }
  L.total = o;
  return L;
}

static int ncu_of(hipStream_t st) {
  int dev = 0, n = 256;
  if (hipStreamGetDevice(st, &dev) != hipSuccess ||
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    n = 256;
  return n >= 8 ? n / 8 * 8 : 8;
}

#define NR_FT(x)                  \
  do {                            \
    const int rc_ = (x);          \
    if (rc_ != NR_OK) return rc_; \
  } while (0)
#define NR_FT_EV(x, what)                                         \
  do {                                                            \
    if ((x) != hipSuccess) {                                      \
      set_error("nr_final_train_step: %s failed", what);          \
      return NR_ERR_HIP;                                          \
    }                                                             \
  } while (0)

template <typename TA>
int step(const nr_final_train_args& a, char* ws, hipStream_t st) {
  constexpr bool BF = sizeof(TA) == 2;
  const int dt = a.dtype;
  const int ncu = ncu_of(st);
  const Layout L = layout(dt, a.B, a.U, a.Hs, ncu);
  const int64_t B = a.B, Hs = a.Hs, Hp = L.Hp;
  auto P_ = [&](int64_t off) { return (void*)(ws + off); };
  float* xpair = (float*)P_(L.xpair);
  TA* XH = (TA*)P_(L.XH);
  TA *S = (TA*)P_(L.S), *X1 = (TA*)P_(L.X1), *X2 = (TA*)P_(L.X2), *XP = (TA*)P_(L.XP), *Y = (TA*)P_(L.Y);
  float* users = a.users ? a.users : (float*)P_(L.users);
  float *z = (float*)P_(L.z), *du = (float*)P_(L.du), *gpair = (float*)P_(L.gpair), *lrow = (float*)P_(L.lrow);
  TA *dXp = (TA*)P_(L.dXp), *dL = (TA*)P_(L.dL), *dY = (TA*)P_(L.dY), *dX = (TA*)P_(L.dX), *dZ2 = (TA*)P_(L.dZ2);
  TA* dZ1 = (TA*)P_(L.dZ1);
  TA *W2t = (TA*)P_(L.W2t), *W3t = (TA*)P_(L.W3t), *W4t = (TA*)P_(L.W4t),
     *W5t = (TA*)P_(L.W5t);
  const TA *W1 = (const TA*)a.W1, *W2 = (const TA*)a.W2, *W3 = (const TA*)a.W3, *W4 = (const TA*)a.W4,
           *W5 = (const TA*)a.W5;
  TA* X = XP;           // [Hp][D] at row stride 2D
  TA* Pexp = XP + D;    // exp(logits), same stride
  const float scale = 1.0f / (1.0f - a.p);
  const uint32_t thr = dropout_threshold(a.p);
  TrainSide side;
  NR_FT(train_side_streams(st, "nr_final_train_step", side));

  // ---- the weight transposes the data-grad GEMMs need, on the side stream beside
  // an N = 1024 forward GEMM (X: 132 tiles, half of the CUs idle) rather than
  // beside the full-chip ones; joined (event wt) before the first data-grad GEMM
  auto transposes = [&](int i0, int i1, hipEvent_t fork) -> int {
    // (no W1^T: its only consumer was the dS = dZ1 W1 GEMM, folded away below)
    const TA* w[4] = {W5, W4, W3, W2};
    TA* t[4] = {W5t, W4t, W3t, W2t};
    const int64_t r[4] = {D, H, D, H}, c[4] = {H, D, H, H};  // W5 [D][H], W4 [H][D], W3 [D][H], W2 [H][H]
    NR_FT_EV(hipEventRecord(fork, st), "fork record");
    NR_FT_EV(hipStreamWaitEvent(side.s, fork, 0), "fork wait");
    for (int i = i0; i < i1; ++i) NR_FT(nr_transpose(dt, dt, r[i], c[i], w[i], c[i], t[i], r[i], side.s));
    return NR_OK;
  };

  // ---- accumulators: f32 mode's bias grads (nr_col_sum adds); everything else is
  // written whole (the loss and token LN grads by ordered sums, no atomics)
  if constexpr (!BF) {
    ZList zl{};
    float* zp[4] = {a.g_b1, a.g_b2, a.g_b3, a.g_b4};
    const int64_t zn[4] = {H, H, D, H};
    zl.n = 4;
    for (int i = 0; i < zl.n; ++i) { zl.p[i] = zp[i]; zl.len[i] = zn[i]; }
    hipLaunchKernelGGL(zero_kernel, dim3(64), dim3(256), 0, st, zl);
    NR_CHECK_LAUNCH("nr_final_train_step (zero)");
  }
  // ---- forward
  // the slots' S and XH: the token LN of each slot's news (one kernel, no [U][D] table)
  {
    const int64_t g = (Hp + 3) / 4;
    const dim3 grid((unsigned)(g < 4096 ? g : 4096));
#define NR_FT_TOK(TT) \
    hipLaunchKernelGGL((slots_kernel<TA, TT>), grid, dim3(256), 0, st, Hp, Hs, (const TT*)a.tok_last, a.hist_idx, \
                       a.tok_g, a.tok_b, S, XH)
    if (a.tok_dtype == NR_F32) NR_FT_TOK(float);
    else if (a.tok_dtype == NR_BF16) NR_FT_TOK(__bf16);
    else NR_FT_TOK(_Float16);
#undef NR_FT_TOK
    NR_CHECK_LAUNCH("nr_final_train_step (slots)");
  }
  // relu(dropout) GEMM over Hp rows: main rows on the persistent kernel, the tail as K-slices + fixup
  auto relu_gemm = [&](const TA* A, int64_t lda, const TA* W, int64_t K, const float* bias, uint64_t seed, TA* C,
                       int64_t ldc) -> int {
    EpiArgs ea{seed, thr, scale};
    const int64_t mm = split_tail(K) ? L.mm : Hp;
    NR_FT(gemm_dispatch_ex(dt, dt, NR_EPI_RELU_DROPOUT, mm, H, K, A, lda, W, K, bias, nullptr, 0, C, ldc, ea, st));
    if (mm == Hp) return NR_OK;
    float* Pk = (float*)P_(L.skP);
    const int ns = kSplit;
    const int64_t kk = K / ns, rows = Hp - mm;
    GemmProblem p = {rows, H, kk, A + mm * lda, lda, kk, W, K, kk, Pk, H, rows * H, ns, 1.0f};
    NR_FT(gemm_group_dispatch(dt, NR_F32, &p, 1, st));
    return nr_splitk_fixup(dt, NR_EPI_RELU_DROPOUT, rows, H, ns, Pk, bias, nullptr, 0, C + mm * ldc, ldc, mm,
                           seed, a.p, scale, st);
  };
  NR_FT(relu_gemm(S, D, W1, D, a.b1, a.seed[0], X1, H));
  NR_FT(relu_gemm(X1, H, W2, H, a.b2, a.seed[1], X2, H));
  // all four beside X under one fork; a second fork for the last ones beside P measured
  // the same (interleaved A/B, profiles/round5/train/ab_r7u)
  NR_FT(transposes(0, 4, side.fork));
  NR_FT_EV(hipEventRecord(side.wt, side.s), "transpose record");
  NR_FT(gemm_dispatch(dt, dt, NR_EPI_NONE, Hp, D, H, X2, H, W3, H, a.b3, nullptr, 0, X, 2 * D, st));
  NR_FT(relu_gemm(X, 2 * D, W4, D, a.b4, a.seed[2], Y, H));
  NR_FT(gemm_dispatch(dt, dt, NR_EPI_EXP, Hp, D, H, Y, H, W5, H, nullptr, nullptr, 0, Pexp, 2 * D, st));
  NR_FT(nr_final_pool_fwd(dt, B, a.hist_off, XP, 2 * D, users, z, st));
  // ---- loss and its gradient into the pooled users and E[pos] / E[neg]
  {
    const dim3 grid((unsigned)((B + 3) / 4));
#define NR_FT_TOK(TT) \
    hipLaunchKernelGGL((cos_pairs_kernel<TT>), grid, dim3(256), 0, st, B, users, (const TT*)a.tok_last, xpair, \
                       a.tok_g, a.tok_b, a.pos, a.neg, a.margin, lrow, du, gpair)
    if (a.tok_dtype == NR_F32) NR_FT_TOK(float);
    else if (a.tok_dtype == NR_BF16) NR_FT_TOK(__bf16);
    else NR_FT_TOK(_Float16);
#undef NR_FT_TOK
  }
  NR_CHECK_LAUNCH("nr_final_train_step (cosine)");
  // the pairs' token LN grad partials (after the W1 fold's chunks) and the loss
  hipLaunchKernelGGL(pair_ln_kernel, dim3((unsigned)(D / 64), kPairChunks), dim3(256), 0, st, B, gpair, xpair, lrow,
                     (float*)P_(L.w1p) + (H / 64) * 2 * D, a.loss);
  NR_CHECK_LAUNCH("nr_final_train_step (pair LN grads)");
  NR_FT(nr_final_pool_bwd(dt, B, a.hist_off, Hp, XP, 2 * D, users, z, du, dXp, D, dL, D, st));
  // ---- data-grad chain (weights transposed on the side stream)
  NR_FT_EV(hipStreamWaitEvent(st, side.wt, 0), "transpose wait");
  float *cs4 = (float*)P_(L.cs4), *cs3 = (float*)P_(L.cs3), *cs2 = (float*)P_(L.cs2), *cs1 = (float*)P_(L.cs1);
  // drop'(A W^T) against the forward output Yf; bf16: column sums into cs
  auto drelu_gemm = [&](const TA* A, int64_t K, const TA* Wt, const TA* Yf, TA* C, float* cs, float* gbias) -> int {
    if constexpr (!BF) {
      NR_FT(gemm_dispatch_ex(dt, dt, NR_EPI_DRELU, Hp, H, K, A, K, Wt, K, nullptr, Yf, H, C, H,
                             EpiArgs{0, 0, scale}, st));
      return nr_col_sum(dt, Hp, H, C, H, gbias, st);
    } else {
      EpiArgs ea{0, 0, scale};
      ea.colsum = cs;
      const int64_t mm = split_tail(K) ? L.mm : Hp;
      NR_FT(gemm_dispatch_ex(dt, dt, NR_EPI_DRELU, mm, H, K, A, K, Wt, K, nullptr, Yf, H, C, H, ea, st));
      if (mm == Hp) return NR_OK;
      float* Pk = (float*)P_(L.skP);
      const int ns = kSplit;
      const int64_t kk = K / ns, rows = Hp - mm;
      GemmProblem p = {rows, H, kk, A + mm * K, K, kk, Wt, K, kk, Pk, H, rows * H, ns, 1.0f};
      NR_FT(gemm_group_dispatch(dt, NR_F32, &p, 1, st));
      // the fixup and the tail rows' column sums (of the stored bf16 values) in one launch
      hipLaunchKernelGGL((fixup_drelu_cs_kernel<TA>), dim3((unsigned)(H / 64), (unsigned)((rows + 31) / 32)),
                         dim3(256), 0, st, mm / 128, rows, H, ns, Pk, Yf + mm * H, H, C + mm * H, H, scale, cs);
      NR_CHECK_LAUNCH("nr_final_train_step (tail fixup + column sums)");
      return NR_OK;
    }
  };
  NR_FT(drelu_gemm(dL, D, W5t, Y, dY, cs4, a.g_b4));  // dY = drop'(dL W5): the grad of linear4's output
  {
    EpiArgs ea{0, 0, 1.f};
    if constexpr (BF) ea.colsum = cs3;
    NR_FT(gemm_dispatch_ex(dt, dt, NR_EPI_RESADD, Hp, D, H, dY, H, W4t, H, nullptr, dXp, D, dX, D, ea, st));
    if constexpr (!BF) NR_FT(nr_col_sum(dt, Hp, D, dX, D, a.g_b3, st));
  }
  NR_FT(drelu_gemm(dX, D, W3t, X2, dZ2, cs2, a.g_b2));
  NR_FT(drelu_gemm(dZ2, H, W2t, X1, dZ1, cs1, a.g_b1));
  // (no dS = dZ1 W1: its only consumer, the token LN parameters, folds into dW1 below)
  // ---- weight grads: dW = dOut^T X
  RSum r{};  // bf16: the bias grads from the column-sum partials
  if constexpr (BF) {
    GemmProblem p[5] = {
        {D, H, Hp, dL, D, 0, Y, H, 0, a.g_W5, H, 0, 1, 1.0f},
        {H, D, Hp, dY, H, 0, X, 2 * D, 0, a.g_W4, D, 0, 1, 1.0f},
        {D, H, Hp, dX, D, 0, X2, H, 0, a.g_W3, H, 0, 1, 1.0f},
        {H, H, Hp, dZ2, H, 0, X1, H, 0, a.g_W2, H, 0, 1, 1.0f},
        {H, D, Hp, dZ1, H, 0, XH, D, 0, a.g_W1, D, 0, 1, 1.0f},  // M = dZ1^T XH (w1_fold_kernel)
    };
    float* sqp = a.sumsq ? (float*)P_(L.sqp) : nullptr;
    const bool sqf[5] = {true, true, true, true, false};  // dW1 is M here: counted by the fold
    // one sum-of-squares slot per tile: the five shapes are fixed, so is the tile count
    static_assert(4 * (D / 256) * (H / 256) + (H / 256) * (H / 256) == kSqTn, "weight-grad tiles != kSqTn");
    NR_FT(gemm_group_tn_dispatch(NR_F32, p, 5, st, sqp, sqf, nullptr, kSqTn));
    float* parts[4] = {cs1, cs2, cs3, cs4};
    float* outs[4] = {a.g_b1, a.g_b2, a.g_b3, a.g_b4};
    const int64_t cols[4] = {H, H, D, H};
    r.n = 4;
    // (cs1: dZ1, K = H, tail split; cs2 / cs4: dZ2 / dY, K = D, and cs3: dX, none)
    static_assert(!split_tail(D) && split_tail(H), "column-sum row counts assume the K = D GEMMs run unsplit");
    const int64_t crows[4] = {L.csr, L.csr3, L.csr3, L.csr3};
    for (int i = 0; i < 4; ++i) { r.part[i] = parts[i]; r.out[i] = outs[i]; r.rows[i] = crows[i]; r.cols[i] = cols[i]; }
    // (launched with the W1 fold below: bias_fold_kernel)
  } else {
    TA* T[10];
    for (int i = 0; i < 10; ++i) T[i] = (TA*)P_(L.T[i]);
    const TA* src[10] = {dL, Y, dY, X, dX, X2, dZ2, X1, dZ1, XH};
    const int64_t cols[10] = {D, H, H, D, D, H, H, H, H, D}, ld[10] = {D, H, H, 2 * D, D, H, H, H, H, D};
    for (int i = 0; i < 10; ++i) NR_FT(nr_transpose(dt, dt, Hp, cols[i], src[i], ld[i], T[i], Hp, st));
    GemmProblem p[5] = {
        {D, H, Hp, T[0], Hp, 0, T[1], Hp, 0, a.g_W5, H, 0, 1, 1.0f},
        {H, D, Hp, T[2], Hp, 0, T[3], Hp, 0, a.g_W4, D, 0, 1, 1.0f},
        {D, H, Hp, T[4], Hp, 0, T[5], Hp, 0, a.g_W3, H, 0, 1, 1.0f},
        {H, H, Hp, T[6], Hp, 0, T[7], Hp, 0, a.g_W2, H, 0, 1, 1.0f},
        {H, D, Hp, T[8], Hp, 0, T[9], Hp, 0, a.g_W1, D, 0, 1, 1.0f},
    };
    NR_FT(gemm_group_dispatch(dt, NR_F32, p, 5, st));
  }
  // ---- token LayerNorm parameter grads: the history gather's part folded with dW1
  // (w1_fold_kernel; dW1 = gamma o M + g_b1 (x) beta), summed with the pairs' part
  // (bf16: one launch with the bias grads)
  {
    float* w1p = (float*)P_(L.w1p);
    float* sqp = BF && a.sumsq ? (float*)P_(L.sqp) : nullptr;
    if constexpr (BF) {
      const int nrs = (int)((3 * H + D) / 64);
      hipLaunchKernelGGL((bias_fold_kernel<TA>), dim3((unsigned)(nrs + (D / 64) * (H / 64))), dim3(256), 0, st, r, nrs,
                         sqp ? sqp + kSqTn + kSqFold : nullptr, W1, a.g_W1, a.tok_g, a.tok_b, w1p,
                         sqp ? sqp + kSqTn : nullptr);
      NR_CHECK_LAUNCH("nr_final_train_step (bias grads + W1 fold)");
    } else {
      hipLaunchKernelGGL((w1_fold_kernel<TA>), dim3((unsigned)(D / 64), (unsigned)(H / 64)), dim3(256), 0, st, W1,
                         a.g_W1, a.g_b1, a.tok_g, a.tok_b, w1p, nullptr);
      NR_CHECK_LAUNCH("nr_final_train_step (W1 fold)");
    }
    hipLaunchKernelGGL(ln_reduce_kernel, dim3((unsigned)(D / 64)), dim3(256), 0, st, (int)(H / 64) + kPairChunks, w1p,
                       a.g_tok_g, a.g_tok_b, sqp ? sqp + kSqTn + kSqFold + kSqBias : nullptr);
    NR_CHECK_LAUNCH("nr_final_train_step (token LN grads)");
    if (sqp) {
      hipLaunchKernelGGL(sq_total_kernel, dim3(1), dim3(256), 0, st, (int64_t)kSqParts, sqp, a.sumsq);
      NR_CHECK_LAUNCH("nr_final_train_step (grad norm)");
    } else if (a.sumsq) {  // f32 mode: over the gradient arrays
      hipLaunchKernelGGL(zero_kernel, dim3(1), dim3(256), 0, st, ZList{{a.sumsq}, {1}, 1});
      NR_CHECK_LAUNCH("nr_final_train_step (zero)");
      float* gs[11] = {a.g_tok_g, a.g_tok_b, a.g_W1, a.g_b1, a.g_W2, a.g_b2, a.g_W3, a.g_b3, a.g_W4, a.g_b4, a.g_W5};
      const int64_t gn[11] = {D, D, H * D, H, H * H, H, D * H, D, H * D, H, D * H};
      for (int i = 0; i < 11; ++i) NR_FT(nr_sumsq(gn[i], gs[i], a.sumsq, st));
    }
  }
  return NR_OK;
}
#undef NR_FT
#undef NR_FT_EV

}  // namespace ft
}  // namespace nr

// (the split-K tail, and so the workspace, depends on the device's CU count:
// sized for the CURRENT device here, checked against the stream's device by the step)
extern "C" int64_t nr_final_train_workspace_bytes(int dtype, int64_t B, int64_t U, int64_t Hs) {
  if ((dtype != NR_F32 && dtype != NR_BF16) || B < 0 || U < 0 || Hs < 0) return -1;
  int dev = 0, n = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    n = 256;
  return nr::ft::layout(dtype, B, U, Hs, n >= 8 ? n / 8 * 8 : 8).total;
}

extern "C" int nr_final_train_step(const nr_final_train_args* args, void* ws, int64_t ws_bytes, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(args, "nr_final_train_step: null args");
  const nr_final_train_args& a = *args;
  NR_CHECK_ARG(a.dtype == NR_F32 || a.dtype == NR_BF16, "nr_final_train_step: dtype must be NR_F32 or NR_BF16");
  NR_CHECK_ARG(a.tok_dtype == NR_F32 || a.tok_dtype == NR_BF16 || a.tok_dtype == NR_F16,
               "nr_final_train_step: bad tok_dtype");
  NR_CHECK_ARG(a.B >= 1 && a.U >= 1 && a.Hs >= 1, "nr_final_train_step: empty batch (B=%lld U=%lld Hs=%lld)",
               (long long)a.B, (long long)a.U, (long long)a.Hs);
  NR_CHECK_ARG(a.Hs <= (1ll << 31) - 1024 && a.U <= (1ll << 31) && a.B <= (1ll << 24),
               "nr_final_train_step: batch too large");
  NR_CHECK_ARG(a.p >= 0.f && a.p < 1.f, "nr_final_train_step: dropout p outside [0, 1)");
  // bf16: the persistent GEMM (the column-sum epilogues have no other kernel) addresses
  // its [Hp][4096] operands through 32-bit buffer offsets; refuse before any launch
  NR_CHECK_ARG(a.dtype != NR_BF16 || nr::ft::pad64(a.Hs) * nr::ft::H * 2 <= 0xFFFFFFFFll,
               "nr_final_train_step: bf16 batch of %lld history slots exceeds the persistent GEMM's 4 GiB operand "
               "range (at most %lld)", (long long)a.Hs, 0xFFFFFFFFll / (2 * nr::ft::H) / 64 * 64);
  NR_CHECK_DEVICE("nr_final_train_step", a.tok_last, a.hist_idx, a.hist_off, a.pos, a.neg, a.tok_g, a.tok_b, a.W1,
                  a.b1, a.W2, a.b2, a.W3, a.b3, a.W4, a.b4, a.W5);
  NR_CHECK_DEVICE("nr_final_train_step", a.g_tok_g, a.g_tok_b, a.g_W1, a.g_b1, a.g_W2, a.g_b2, a.g_W3, a.g_b3, a.g_W4,
                  a.g_b4, a.g_W5, a.loss, a.users, a.sumsq, ws);
  NR_CHECK_ARG(a.tok_last && a.hist_idx && a.hist_off && a.pos && a.neg && a.loss && ws && a.tok_g && a.tok_b &&
                   a.W1 && a.b1 && a.W2 && a.b2 && a.W3 && a.b3 && a.W4 && a.b4 && a.W5 && a.g_W1 && a.g_W2 && a.g_W3 && a.g_W4 && a.g_W5 && a.g_b1 && a.g_b2 && a.g_b3 &&
                   a.g_b4 && a.g_tok_g && a.g_tok_b,
               "nr_final_train_step: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int64_t need = nr::ft::layout(a.dtype, a.B, a.U, a.Hs, nr::ft::ncu_of(s)).total;
  NR_CHECK_ARG(ws_bytes >= need, "nr_final_train_step: workspace too small (%lld < %lld)", (long long)ws_bytes,
               (long long)need);
  NR_CHECK_ARG(((uintptr_t)ws & 255) == 0, "nr_final_train_step: workspace must be 256-byte aligned");
  return a.dtype == NR_F32 ? nr::ft::step<float>(a, (char*)ws, s) : nr::ft::step<__bf16>(a, (char*)ws, s);
}
