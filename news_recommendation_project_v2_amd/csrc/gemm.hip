// MFMA GEMMs with fused epilogues for the per-news pooler transforms (gfx950).
//
//   C[M, N] = epilogue(A[M, K] · W[N, K]ᵀ)     (W in torch nn.Linear layout)
//
// Replaces nn.Linear (+ F.relu / torch.exp / GEGLU / residual add) in
//   FinalAttention.forward        modeling_utils.py:218-222
//   LatentAttentionModel blocks   latent_attention.py:34-36, 59-61, 162-163
//
// Two main loops share one tiling and one epilogue:
//   f32 : v_mfma_f32_32x32x2_f32  (exact f32 fmaf chain; the parity config)
//   bf16: v_mfma_f32_32x32x16_bf16 (bf16 operands, f32 accumulate)
// Block tile 128x128, 256 threads = 4 waves in a 2x2 grid, each wave owns a
// 64x64 output = 2x2 MFMA 32x32 accumulators (64 acc registers).  K is staged
// through LDS in 128-byte row slices (BK = 32 f32 / 64 bf16) with a 16-byte
// row pad (144-byte rows) so the ds_read_b128 fragment reads of 32 distinct
// rows are bank-conflict free; global->register prefetch of tile k+1 overlaps
// the MFMAs of tile k, one barrier per K tile.
#include "nr_common.h"

#include <atomic>


namespace nr {

constexpr int GBM = 128, GBN = 128;
constexpr int GROW = 36;  // LDS row stride in 32-bit words (128 B data + 16 B pad)

// Exact-erf GELU, 0.5 g (1 + erf(g / sqrt 2)) (F.gelu default: latent_attention.py:27,
// XLM-R hidden_act "gelu"), written through erfc(z) = t exp(-z^2 + P(t)),
// t = 1 / (1 + z / 2) (Numerical Recipes erfcc: fractional error < 1.2e-7
// everywhere).  Branch-free: ~16 VALU ops instead of the divergent two-range
// erff, which dominated the GEGLU epilogue.  |gelu - exact| <= 6.1e-7 for
// |g| <= 12 (checked in float64), i.e. f32 rounding level.
__device__ __forceinline__ float gelu_erf(float g) {
  const float x = g * 0.70710678118654752440f;
  const float z = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  const float ans = t * __expf(fmaf(t, p, fmaf(-z, z, -1.26551223f)));  // erfc(|x|)
  return x >= 0.f ? g * fmaf(-0.5f, ans, 1.0f) : 0.5f * g * ans;
}

// exp of the persistent bf16 kernel's EXP and SOFTMAX64 epilogues: v_exp_f32 of
// x log2(e) (relative error ~1e-6 here, against bf16 outputs' 2^-8), not the
// range-reduced expf (13 instructions): the softmax64 epilogue was 13.5 k
// cycles per tile against 4.2 k for a plain one; S GEMM 745 -> 874 TF/s,
// FinalAttention transform -2.4 % (round 3, profiles/round3/s4/).  The f32
// parity kernels keep expf.
__device__ __forceinline__ float epi_exp(float x) { return __expf(x); }

// gelu_erf2x2 (the persistent bf16 kernel's GELU / GEGLU epilogues): nr_common.h.

// EpiArgs (dropout / LN-fold / column-sum arguments of the epilogues): nr_common.h.

template <typename TO>
__device__ __forceinline__ TO to_out(float v) {
  if constexpr (sizeof(TO) == 4) return v; else return (TO)v;
}
template <typename TO>
__device__ __forceinline__ float from_out(TO v) {
  if constexpr (sizeof(TO) == 4) return v; else return (float)v;
}

// acc[mi][ni]: 32x32 tile at rows wrow + 32 mi, cols wcol + 32 ni.
// C/D map (gfx950, dtype independent): col = lane & 31,
// row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5).
template <int EPI, typename TO>
__device__ __forceinline__ void gemm_epilogue(const f32x16 (&acc)[2][2], int64_t M, int64_t wrow,
                                              int64_t wcol, int lane, const float* __restrict__ bias,
                                              const TO* R, int64_t ldr, TO* C, int64_t ldc,
                                              int64_t N, const EpiArgs& ea) {
  const int cl = lane & 31;
  const int rh = 4 * (lane >> 5);
  if constexpr (EPI == NR_EPI_GEGLU) {
    // ni = 0 holds the 32 "a" columns, ni = 1 the matching 32 "g" columns.
    const int64_t ca = wcol + cl, cg = wcol + 32 + cl;
    const float ba = bias ? bias[ca] : 0.f, bg = bias ? bias[cg] : 0.f;
    const int64_t oc = wcol / 2 + cl;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int64_t row = wrow + 32 * mi + (reg & 3) + 8 * (reg >> 2) + rh;
        if (row < M) {
          const float a = acc[mi][0][reg] + ba;
          const float g = acc[mi][1][reg] + bg;
          C[row * ldc + oc] = to_out<TO>(a * gelu_erf(g));
        }
      }
    }
  } else {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int64_t col = wcol + 32 * ni + cl;
      const float b = bias ? bias[col] : 0.f;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int64_t row = wrow + 32 * mi + (reg & 3) + 8 * (reg >> 2) + rh;
          if (row < M) {
            float v = acc[mi][ni][reg] + b;
            if constexpr (EPI == NR_EPI_RELU) v = fmaxf(v, 0.f);
            if constexpr (EPI == NR_EPI_RELU_DROPOUT)
              v = drop_at(ea.seed, (uint64_t)(row * N + col), ea.thr) ? 0.f : fmaxf(v, 0.f) * ea.scale;
            if constexpr (EPI == NR_EPI_EXP) v = expf(v);
            if constexpr (EPI == NR_EPI_GELU) v = gelu_erf(v);
            if constexpr (EPI == NR_EPI_RESADD) v += from_out<TO>(R[row * ldr + col]);
            if constexpr (EPI == NR_EPI_DRELU) v = from_out<TO>(R[row * ldr + col]) > 0.f ? v * ea.scale : 0.f;
            C[row * ldc + col] = to_out<TO>(v);
          }
        }
      }
    }
  }
}

// TI = float (f32 MFMA, BK = 32) or __bf16 (bf16 MFMA, BK = 64).  A row slice
// of one K tile is always 128 bytes = 8 x 16-byte chunks.
template <typename TI, int EPI, typename TO>
__global__ __launch_bounds__(256, 2) void gemm_kernel(int64_t M, int64_t N, int64_t K,
                                                      const TI* __restrict__ A, int64_t lda,
                                                      const TI* __restrict__ W, int64_t ldw,
                                                      const float* __restrict__ bias, const TO* R,
                                                      int64_t ldr, TO* C, int64_t ldc, EpiArgs ea) {
  constexpr int BK = 128 / (int)sizeof(TI);
  constexpr int TILE_WORDS = GBM * GROW;  // one operand tile, 32-bit words
  __shared__ __attribute__((aligned(16))) uint32_t smem[2 * 2 * TILE_WORDS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t n0 = (int64_t)blockIdx.x * GBN;
  const int64_t m0 = (int64_t)blockIdx.y * GBM;

  // global -> register staging map: 4 chunks of 16 B per operand per thread
  int srow[4], schk[4];
  const uint4* ga[4];
  const uint4* gw[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int id = tid + 256 * p;
    srow[p] = id >> 3;
    schk[p] = id & 7;
    const int64_t ar = min(m0 + srow[p], M - 1);
    ga[p] = reinterpret_cast<const uint4*>(A + ar * lda) + schk[p];
    gw[p] = reinterpret_cast<const uint4*>(W + (n0 + srow[p]) * ldw) + schk[p];
  }
  const int64_t kstep16 = BK * (int64_t)sizeof(TI) / 16;  // 16-B chunks per K tile = 8

  uint4 ra[4], rw[4];
  auto gload = [&](int64_t kt) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      ra[p] = ga[p][kt * kstep16];
      rw[p] = gw[p][kt * kstep16];
    }
  };
  auto lstore = [&](int buf) {
    uint32_t* As = smem + buf * 2 * TILE_WORDS;
    uint32_t* Ws = As + TILE_WORDS;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      *reinterpret_cast<uint4*>(As + srow[p] * GROW + schk[p] * 4) = ra[p];
      *reinterpret_cast<uint4*>(Ws + srow[p] * GROW + schk[p] * 4) = rw[p];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
  const int arow0 = (wm * 64 + fr) * GROW, wrow0 = (wn * 64 + fr) * GROW;

  auto compute = [&](int buf) {
    const uint32_t* As = smem + buf * 2 * TILE_WORDS;
    const uint32_t* Ws = As + TILE_WORDS;
    if constexpr (sizeof(TI) == 4) {
      // lane half h covers k = 16h + 4q + t of the 32-deep tile (A and W alike)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4 af[2], wf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          af[i] = *reinterpret_cast<const f32x4*>(As + arow0 + 32 * i * GROW + 16 * fh + 4 * q);
          wf[i] = *reinterpret_cast<const f32x4*>(Ws + wrow0 + 32 * i * GROW + 16 * fh + 4 * q);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi][t], wf[ni][t], acc[mi][ni], 0, 0, 0);
      }
    } else {
      // lane (r, h) holds k = 16ks + 8h + j, j < 8, of row r (32x32x16 operand map)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8 af[2], wf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          af[i] = *reinterpret_cast<const bf16x8*>(As + arow0 + 32 * i * GROW + 8 * ks + 4 * fh);
          wf[i] = *reinterpret_cast<const bf16x8*>(Ws + wrow0 + 32 * i * GROW + 8 * ks + 4 * fh);
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], wf[ni], acc[mi][ni], 0, 0, 0);
      }
    }
  };

  const int64_t nk = K / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = (int)(kt & 1);
    if (kt + 1 < nk) gload(kt + 1);
    compute(cur);
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  gemm_epilogue<EPI, TO>(acc, M, m0 + wm * 64, n0 + wn * 64, lane, bias, R, ldr, C, ldc, N, ea);
}

// ---------------------------------------------------------------------------
// bf16, 256x256 block tile, 512 threads = 8 waves (2 along M x 4 along N),
// each wave 128x64 = 4x2 accumulators of 32x32 (128 acc VGPRs).  K tiles of
// 64 are staged global -> LDS directly with global_load_lds_dwordx4 (no VGPR
// round trip) into a 2-stage ring (2 x 64 KiB); the prefetch of tile k+1 is in
// flight while the MFMAs of tile k run, one barrier per K tile.  LDS image of
// an operand stage: row r (0..255) = 8 chunks of 16 B, chunk c stored at
// position c ^ ((r >> 1) & 7): each 16-lane ds_read_b128 group then hits 16
// distinct 16-B bank slots (T2 swizzle, applied on the glds SOURCE address
// because the DMA writes LDS lane-linearly).
constexpr int G2BM = 256, G2BN = 256;
constexpr int G2_STAGE = (G2BM + G2BN) * 128;  // bytes per stage (A + B, 128-B row slices) = 64 KiB

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void g_void;

// Epilogue of the 256x256 kernels (acc[4][2] per wave: rows wm*128 + 32 mi,
// cols wn*64 + 32 ni), staged through the kernel's LDS (caller has finished
// with the operand stages and passed a barrier).
template <bool MF16>
struct Acc256 {  // per-wave 128x64 accumulators: 4x2 tiles of 32x32, or 8x4 tiles of 16x16
  typedef f32x16 type[4][2];
};
template <>
struct Acc256<true> {
  typedef f32x4 type[8][4];
};

template <int EPI, typename TO, bool MF16 = false>
__device__ __forceinline__ void gemm256_store(const typename Acc256<MF16>::type& acc, unsigned char* smem, int wave, int lane,
                                              int wm, int wn, int64_t m0, int64_t n0, int64_t M, int64_t N,
                                              const float* __restrict__ bias, const TO* R, int64_t ldr, TO* C,
                                              int64_t ldc, const EpiArgs& ea) {
  // Epilogue, staged through LDS so global stores are whole 16-byte row
  // segments (the 32x32 C/D map would give 2-4-byte scattered stores).  Two
  // passes of 64 rows per wave; bias and activation are applied in registers,
  // the f32 results parked in the wave's private 16 KiB LDS slab
  // ([64 rows][COLS] f32), then read back row-wise, residual added, stored.
  constexpr int COLS = (EPI == NR_EPI_GEGLU) ? 32 : 64;  // output columns per wave
  constexpr int VEC = 16 / (int)sizeof(TO);               // elements per 16-B store
  constexpr int LPR = COLS / VEC;                          // lanes per output row
  constexpr int RPI = 64 / LPR;                            // rows per wave instruction
  const int cl = lane & 31, rh = 4 * (lane >> 5);
  float* slab = reinterpret_cast<float*>(smem + wave * 16384);
  float sq = 0.f;  // ea.sq_part: this thread's sum of squares of the values it stores
  // The slabs overlay the operand stages: one workgroup barrier so that no
  // wave still reads operands; after it each wave only touches its own slab,
  // so the passes order their LDS traffic wave-locally (no further workgroup
  // barriers: waves drift apart and their store bursts spread out).
  __syncthreads();
#define NR_EPI_SYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
  const int64_t wcol = n0 + wn * 64;
  const int64_t ocol0 = (EPI == NR_EPI_GEGLU) ? wcol / 2 : wcol;
  float ba = 0.f, bg = 0.f;
  float b16[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (MF16) {
    if (bias) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) b16[ni] = bias[wcol + 16 * ni + (lane & 15)];
    }
  } else if (bias) {
    ba = bias[wcol + cl];
    bg = bias[wcol + 32 + cl];
  }
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if constexpr (MF16) {
      // 16x16 C/D map: col = lane & 15, row = 4 * (lane >> 4) + r
      const int c16 = lane & 15, r16 = 4 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mi = 4 * pass + i;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = 16 * i + r16 + r;
          if constexpr (EPI == NR_EPI_GEGLU) {
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              slab[lr * COLS + 16 * ni + c16] = (acc[mi][ni][r] + b16[ni]) * gelu_erf(acc[mi][ni + 2][r] + b16[ni + 2]);
          } else {
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
              float v = acc[mi][ni][r] + b16[ni];
              if constexpr (EPI == NR_EPI_NONE) v *= ea.scale;
              if constexpr (EPI == NR_EPI_RELU) v = fmaxf(v, 0.f);
              if constexpr (EPI == NR_EPI_RELU_DROPOUT) {
                const uint64_t gi = (uint64_t)((m0 + wm * 128 + pass * 64 + lr) * N + wcol + 16 * ni + c16);
                v = drop_at(ea.seed, gi, ea.thr) ? 0.f : fmaxf(v, 0.f) * ea.scale;
              }
              if constexpr (EPI == NR_EPI_EXP) v = expf(v);
              if constexpr (EPI == NR_EPI_GELU) v = gelu_erf(v);
              slab[lr * COLS + 16 * ni + c16] = v;
            }
          }
        }
      }
    } else
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int mi = 2 * pass + h;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int lr = 32 * h + (reg & 3) + 8 * (reg >> 2) + rh;
        if constexpr (EPI == NR_EPI_GEGLU) {
          slab[lr * COLS + cl] = (acc[mi][0][reg] + ba) * gelu_erf(acc[mi][1][reg] + bg);
        } else {
          float v0 = acc[mi][0][reg] + ba, v1 = acc[mi][1][reg] + bg;
          if constexpr (EPI == NR_EPI_NONE) { v0 *= ea.scale; v1 *= ea.scale; }
          if constexpr (EPI == NR_EPI_RELU) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); }
          if constexpr (EPI == NR_EPI_RELU_DROPOUT) {
            const uint64_t gi = (uint64_t)((m0 + wm * 128 + pass * 64 + lr) * N + wcol + cl);
            v0 = drop_at(ea.seed, gi, ea.thr) ? 0.f : fmaxf(v0, 0.f) * ea.scale;
            v1 = drop_at(ea.seed, gi + 32, ea.thr) ? 0.f : fmaxf(v1, 0.f) * ea.scale;
          }
          if constexpr (EPI == NR_EPI_EXP) { v0 = expf(v0); v1 = expf(v1); }
          if constexpr (EPI == NR_EPI_GELU) { v0 = gelu_erf(v0); v1 = gelu_erf(v1); }
          slab[lr * COLS + cl] = v0;
          slab[lr * COLS + 32 + cl] = v1;
        }
      }
    }
    NR_EPI_SYNC();
    const int rr = lane / LPR, cc = (lane % LPR) * VEC;
#pragma unroll
    for (int it = 0; it < 64 / RPI; ++it) {
      const int lr = it * RPI + rr;
      const int64_t row = m0 + wm * 128 + pass * 64 + lr;
      float v[VEC];
#pragma unroll
      for (int q = 0; q < VEC; q += 4) {
        const float4 f = *reinterpret_cast<const float4*>(slab + lr * COLS + cc + q);
        v[q] = f.x; v[q + 1] = f.y; v[q + 2] = f.z; v[q + 3] = f.w;
      }
      if constexpr (EPI == NR_EPI_SOFTMAX64) {
        // the wave's 64 columns are one 64-wide softmax group (column block
        // wn * 64); a row's values sit on LPR consecutive lanes
        float m = v[0];
#pragma unroll
        for (int q = 1; q < VEC; ++q) m = fmaxf(m, v[q]);
#pragma unroll
        for (int o = 1; o < LPR; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        float sum = 0.f;
#pragma unroll
        for (int q = 0; q < VEC; ++q) { v[q] = expf(v[q] - m); sum += v[q]; }
#pragma unroll
        for (int o = 1; o < LPR; o <<= 1) sum += __shfl_xor(sum, o, 64);
        const float inv = 1.0f / sum;
#pragma unroll
        for (int q = 0; q < VEC; ++q) v[q] *= inv;
      }
      if (row < M) {
        if constexpr (EPI == NR_EPI_RESADD || EPI == NR_EPI_DRELU) {
          const uint4 rv = *reinterpret_cast<const uint4*>(R + row * ldr + ocol0 + cc);
          float r[VEC];
          if constexpr (sizeof(TO) == 4) {
            r[0] = __uint_as_float(rv.x); r[1] = __uint_as_float(rv.y);
            r[2] = __uint_as_float(rv.z); r[3] = __uint_as_float(rv.w);
          } else {
            const uint32_t w4[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) { r[2 * q] = bf16_lo(w4[q]); r[2 * q + 1] = bf16_hi(w4[q]); }
          }
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            if constexpr (EPI == NR_EPI_RESADD) v[q] += r[q];
            else v[q] = r[q] > 0.f ? v[q] * ea.scale : 0.f;
          }
        }
        TO o[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) o[q] = to_out<TO>(v[q]);
        *reinterpret_cast<uint4*>(C + row * ldc + ocol0 + cc) = *reinterpret_cast<const uint4*>(o);
        if (ea.sq_part) {
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            const float f = from_out<TO>(o[q]);
            sq = fmaf(f, f, sq);
          }
        }
      }
    }
    NR_EPI_SYNC();
  }
#undef NR_EPI_SYNC
  if (ea.sq_part) {  // workgroup-uniform: the tile's sum of squares (the training step's grad norm)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) sq += __shfl_xor(sq, o, 64);
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    if (lane == 0) red[wave] = sq;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int w = 0; w < 8; ++w) t += red[w];
      ea.sq_part[blockIdx.x] = ea.sq_on ? t : 0.f;
    }
  }
}

// ---------------------------------------------------------------------------
// Pipelined 256x256 variant: each K tile is computed in 4 phases, one output
// quadrant (64 rows x 32 cols per wave) each, with the half-tile LDS-DMA
// prefetches spread over the phases and kept in flight ACROSS raw s_barriers
// (counted vmcnt, never a drained queue in steady state):
//   P1: read A(m0) + B(n0) frags, DMA A-half 0 of tile t+1 -> MFMA q(m0,n0)
//   P2: read B(n1) frags,         DMA A-half 1 of tile t+1 -> MFMA q(m0,n1)
//   P3: read A(m1) frags,         DMA B-half 0 of tile t+2 -> MFMA q(m1,n1)
//   P4: (frags in registers),     DMA B-half 1 of tile t+2 -> MFMA q(m1,n0)
//       (vmcnt(2) before P4's first barrier: tile t+1 has landed)
// A stage's B halves are last read in P2 and its A halves in P3, so the
// prefetch into a stage never overwrites data a wave can still read (each
// phase ends lgkmcnt(0) + barrier).  Block ids are remapped XCD-aware so the
// N-tiles that share an A panel run on one XCD (its L2 holds the panel).
// LDS images: rows of 128 B, chunk c of row r at c ^ ((r >> 1) & 7) (T2 swizzle on the DMA source).
// XCD-aware bijective remap of the launch order: dispatch slot `orig` runs on
// XCD orig % 8; consecutive output tiles (the N tiles sharing an A panel) are
// given to one XCD so its L2 holds the panel.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
  return (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
}

// Output tile of remapped id wg (an XCD runs a contiguous run of ids, ~32 at
// a time).  gm = 1: row-major (the run shares one A panel and reads 32
// different W panels, so at N = 8192 every W slice comes from beyond L2);
// gm > 1: ids go column-major inside groups of gm M-tiles, so a run of 32
// covers gm x 32/gm tiles and each A and W K-slice is fetched into the XCD's
// L2 once for 32/gm resp. gm tiles (miss bytes per tile K-step
// 32 KiB / (32/gm) + 32 KiB / gm instead of 32 KiB / 32 + 32 KiB).
__device__ __forceinline__ void tile_of(int wg, int nx, int ny, int gm, int& mt, int& nt) {
  if (gm <= 1) {
    mt = wg / nx;
    nt = wg % nx;
    return;
  }
  const int per = gm * nx, g = wg / per, first = g * gm;
  const int gsz = min(gm, ny - first), loc = wg - g * per;
  mt = first + loc % gsz;
  nt = loc / gsz;
}

// TN = true (bf16, 16x16x32 only): both operands are stored with the reduction
// index as the ROW, A as [K][M] and W as [K][N] (lda / ldw = their row strides):
// C[m][n] = sum_k A[k][m] W[k][n], i.e. the weight-grad GEMM dW = dOut^T X of a
// training step read straight from the row-major activations dOut [slots][out]
// and X [slots][in], with no transposed copies.  A stage's operand image is
// then two halves (h = tile columns 128 h .. +127) of 64 K-rows x 256 B; the
// 16-B chunk at position P of K-row r holds the row's global chunk
// P ^ (hsw(r) << 1), hsw(r) = (r & 3) | ((r >> 3) & 1) << 2 (applied on the
// DMA source: the DMA writes LDS lane-linearly).  Fragments are read with
// ds_read_b64_tr_b16 (cdna_hip_programming.md T10): lane 4q + p of 16-lane
// group g addresses K-row 8g + 4e + q, columns 4p .. 4p + 3 of its 16-column
// tile and receives its own column's 4 K values, two reads (e = 0, 1) forming
// the 8-deep operand of one 16x16x32 MFMA.  The 8 K-rows a 32-lane half reads
// have distinct hsw, so their 32-B pieces fall in 8 distinct 32-B bank groups
// of the 256-B row: conflict-free.  Host: M % 256 = N % 256 = K % 64 = 0.
__device__ __forceinline__ int tn_hsw(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
typedef short s16x4 __attribute__((ext_vector_type(4)));

template <typename TI, int EPI, typename TO, bool MF16, bool TN = false>
__device__ __forceinline__ void gemm256p_body(unsigned char* smem, int64_t m0, int64_t n0, int64_t M, int64_t N,
                                              int64_t K, const TI* __restrict__ A, int64_t lda,
                                              const TI* __restrict__ W, int64_t ldw, const float* __restrict__ bias,
                                              const TO* R, int64_t ldr, TO* C, int64_t ldc, const EpiArgs& ea) {
  static_assert(!TN || (MF16 && sizeof(TI) == 2), "TN operands: bf16 16x16x32 only");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;

  constexpr int BK = 128 / (int)sizeof(TI), CE = 16 / (int)sizeof(TI);
  // half-tile DMA sources: wave covers rows 128h + 16 wave + 8 j + lane / 8
  // (TN: K-rows 4 (2 wave + j) + lane / 16 of column half h, 16-B position lane & 15)
  const TI* asrc[2][2];
  const TI* bsrc[2][2];
  int hoff[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (TN) {
        const int r = 4 * (wave * 2 + j) + (lane >> 4);
        const int c = (lane & 15) ^ (tn_hsw(r) << 1);
        asrc[h][j] = A + (int64_t)r * lda + m0 + 128 * h + c * CE;
        bsrc[h][j] = W + (int64_t)r * ldw + n0 + 128 * h + c * CE;
        hoff[h][j] = h * 16384 + (wave * 2 + j) * 1024;
      } else {
        const int r0 = 128 * h + (wave * 2 + j) * 8;
        const int row = r0 + (lane >> 3);
        const int chunk = (lane & 7) ^ ((row >> 1) & 7);
        asrc[h][j] = A + min(m0 + row, M - 1) * lda + chunk * CE;
        bsrc[h][j] = W + (n0 + row) * ldw + chunk * CE;
        hoff[h][j] = r0 * 128;
      }
    }
  const int64_t astep = TN ? BK * lda : BK, bstep = TN ? BK * ldw : BK;
  auto dmaA = [&](int h, int stage, int64_t kt) {
    unsigned char* sa = smem + stage * G2_STAGE;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((g_void*)(asrc[h][j] + kt * astep), (lds_void*)(sa + hoff[h][j]), 16, 0, 0);
  };
  auto dmaB = [&](int h, int stage, int64_t kt) {
    unsigned char* sb = smem + stage * G2_STAGE + G2BM * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((g_void*)(bsrc[h][j] + kt * bstep), (lds_void*)(sb + hoff[h][j]), 16, 0, 0);
  };

  typename Acc256<MF16>::type acc;
  if constexpr (MF16) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[mi][ni][r] = 0.f;
  } else {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
  }

  const int fr = lane & 31, fh = lane >> 5;
  // 32x32 operand tiles (MF16 = false): 4 A tiles of 32 rows, 2 B tiles of 32 columns
  // 16x16 operand tiles (MF16 = true):  8 A tiles of 16 rows, 4 B tiles of 16 columns
  constexpr int TA = MF16 ? 8 : 4, TB = MF16 ? 4 : 2, TR = MF16 ? 16 : 32;
  const int lr_ = MF16 ? (lane & 15) : fr;
  int aoff[TA], boff[TB], asw[TA], bsw[TB];
#pragma unroll
  for (int mi = 0; mi < TA; ++mi) {
    const int row = wm * 128 + mi * TR + lr_;
    aoff[mi] = row * 128;
    asw[mi] = (row >> 1) & 7;
  }
#pragma unroll
  for (int ni = 0; ni < TB; ++ni) {
    const int row = wn * 64 + ni * TR + lr_;
    boff[ni] = G2BM * 128 + row * 128;
    bsw[ni] = (row >> 1) & 7;
  }
  // fragment f of a 128-byte row slice:
  //   bf16 32x32x16 k-step f (4 per tile) -> chunk 2f + (lane >> 5)
  //   bf16 16x16x32 k-step f (2 per tile) -> chunk 4f + (lane >> 4)
  //   f32  32x32x2 group f (4 k-steps)    -> chunk 4 (lane >> 5) + f
  auto chunk_of = [&](int f) {
    if constexpr (MF16) return 4 * f + (lane >> 4);
    else return sizeof(TI) == 2 ? 2 * f + fh : 4 * fh + f;
  };
  typedef f32x4 frag_t;  // 16 bytes: 8 bf16 or 4 f32
  constexpr int QA = MF16 ? 4 : 2;   // A tiles per 64-row quadrant
  constexpr int QB = MF16 ? 2 : 1;   // B tiles per 32-column quadrant
  constexpr int NF = MF16 ? 2 : 4;   // fragments (k-steps or groups) per tile per K tile
  frag_t fa[QA][NF], fb0[QB][NF], fb1[QB][NF];
  // TN: per-tile lane offsets of the transposed reads (K-half f adds 8192, e = 1 adds 1024)
  int taoff[TA], tboff[TB];
  if constexpr (TN) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, hsw = q | ((g & 1) << 2);
    const int lrow = (8 * g + q) * 256 + 16 * (p >> 1) + 8 * (p & 1);
#pragma unroll
    for (int mi = 0; mi < TA; ++mi) taoff[mi] = wm * 16384 + lrow + 32 * (mi ^ hsw);
#pragma unroll
    for (int ni = 0; ni < TB; ++ni) {
      const int nrel = wn * 64 + 16 * ni;
      tboff[ni] = G2BM * 128 + (nrel >> 7) * 16384 + lrow + 32 * (((nrel & 127) >> 4) ^ hsw);
    }
  }
  auto tr_frag = [&](const unsigned char* b) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(b));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(b + 1024));
    return __builtin_bit_cast(frag_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto readA = [&](int stage, int qm) {
    const unsigned char* s = smem + stage * G2_STAGE;
#pragma unroll
    for (int i = 0; i < QA; ++i)
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        if constexpr (TN) fa[i][f] = tr_frag(s + taoff[QA * qm + i] + f * 8192);
        else fa[i][f] = *reinterpret_cast<const frag_t*>(s + aoff[QA * qm + i] + ((chunk_of(f) ^ asw[QA * qm + i]) << 4));
      }
  };
  auto readB = [&](int stage, int qn, frag_t (&fb)[QB][NF]) {
    const unsigned char* s = smem + stage * G2_STAGE;
#pragma unroll
    for (int j = 0; j < QB; ++j)
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        if constexpr (TN) fb[j][f] = tr_frag(s + tboff[QB * qn + j] + f * 8192);
        else fb[j][f] = *reinterpret_cast<const frag_t*>(s + boff[QB * qn + j] + ((chunk_of(f) ^ bsw[QB * qn + j]) << 4));
      }
  };
  auto mma = [&](int qm, int qn, const frag_t (&fb)[QB][NF]) {
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int i = 0; i < QA; ++i)
#pragma unroll
        for (int j = 0; j < QB; ++j) {
          if constexpr (MF16) {
            acc[QA * qm + i][QB * qn + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, fa[i][f]), __builtin_bit_cast(bf16x8, fb[j][f]), acc[QA * qm + i][QB * qn + j],
                0, 0, 0);
          } else if constexpr (sizeof(TI) == 2) {
            acc[QA * qm + i][QB * qn + j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                __builtin_bit_cast(bf16x8, fa[i][f]), __builtin_bit_cast(bf16x8, fb[j][f]), acc[QA * qm + i][QB * qn + j],
                0, 0, 0);
          } else {
#pragma unroll
            for (int t = 0; t < 4; ++t)
              acc[QA * qm + i][QB * qn + j] =
                  __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][f][t], fb[j][f][t], acc[QA * qm + i][QB * qn + j], 0, 0, 0);
          }
        }
  };
#define NR_PHASE_SYNC_MMA(QM, NI, FB)                   \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
  __builtin_amdgcn_sched_barrier(0);                   \
  __builtin_amdgcn_s_barrier();                        \
  __builtin_amdgcn_s_setprio(1);                       \
  mma(QM, NI, FB);                                     \
  __builtin_amdgcn_s_setprio(0);                       \
  __builtin_amdgcn_s_barrier();

  // The two wave groups (wm = 0: waves 0-3, wm = 1: waves 4-7; one of each per
  // SIMD) run one barrier apart, so one group's MFMA cluster overlaps the
  // other's fragment reads.  Hazard bookkeeping for that stagger: reads are
  // retired before each phase's first barrier; the tile t+1 landing wait
  // (vmcnt) sits before P4's FIRST barrier so that the leading group, which
  // starts reading tile t+1 one barrier after that, sees the lagging group's
  // DMAs landed too.
  const int wmu = __builtin_amdgcn_readfirstlane(wm);
  const int64_t nk = K / BK;
  dmaB(0, 0, 0);
  dmaB(1, 0, 0);
  dmaA(0, 0, 0);
  dmaA(1, 0, 0);
  if (nk > 1) {
    dmaB(0, 1, 1);
    dmaB(1, 1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wmu == 1) __builtin_amdgcn_s_barrier();  // stagger
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int st = (int)(kt & 1), ns = st ^ 1;
    const bool pre1 = kt + 1 < nk, pre2 = kt + 2 < nk;
    // P1
    readA(st, 0);
    readB(st, 0, fb0);
    if (pre1) dmaA(0, ns, kt + 1);
    NR_PHASE_SYNC_MMA(0, 0, fb0)
    // P2
    readB(st, 1, fb1);
    if (pre1) dmaA(1, ns, kt + 1);
    NR_PHASE_SYNC_MMA(0, 1, fb1)
    // P3
    readA(st, 1);
    if (pre2) dmaB(0, st, kt + 2);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    // P4: tile t+1 must have landed (B0 of t+2 may still fly)
    if (pre2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (pre2) dmaB(1, st, kt + 2);
    __builtin_amdgcn_s_setprio(1);
    mma(1, 0, fb0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  }
  if (wmu == 0) __builtin_amdgcn_s_barrier();  // re-align the groups
#undef NR_PHASE_SYNC_MMA
  gemm256_store<EPI, TO, MF16>(acc, smem, wave, lane, wm, wn, m0, n0, M, N, bias, R, ldr, C, ldc, ea);
}

template <typename TI, int EPI, typename TO, bool MF16 = false>
__global__ __launch_bounds__(512, 2) void gemm256p_kernel(int64_t M, int64_t N, int64_t K,
                                                          const TI* __restrict__ A, int64_t lda,
                                                          const TI* __restrict__ W, int64_t ldw,
                                                          const float* __restrict__ bias, const TO* R,
                                                          int64_t ldr, TO* C, int64_t ldc, EpiArgs ea) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * G2_STAGE];
  const int nx = (int)gridDim.x;
  const int wg = xcd_remap((int)blockIdx.y * nx + (int)blockIdx.x, nx * (int)gridDim.y);
  int mt, nt;
  tile_of(wg, nx, (int)gridDim.y, ea.group_m, mt, nt);
  gemm256p_body<TI, EPI, TO, MF16>(smem, (int64_t)mt * G2BM, (int64_t)nt * G2BN, M, N, K, A, lda, W,
                                   ldw, bias, R, ldr, C, ldc, ea);
}

// Grouped launch of up to kGroupMax independent problems with one dtype pair
// and no bias / residual: one grid over all problems' tiles, so small
// problems (the config-5 weight-grad GEMMs, 64 tiles each) fill the 256 CUs
// together instead of one after another.  A problem may be a strided batch
// (`batch` instances at A + b sA, W + b sW, C + b sC: the 8 heads of the latent
// K/V fold, or the K-slices of a split-K GEMM) and carries a scale alpha
// (C = alpha A W^T).  tile_end[p] = prefix sum of the problems' tile counts
// (tiles x batch); tiles are remapped XCD-aware over the whole grid, so one
// problem's N tiles of an A panel stay on one XCD.
struct GemmGroup {
  int n;
  int tile_end[kGroupMax];
  int ntn[kGroupMax];
  int tpb[kGroupMax];  // tiles per batch instance
  float alpha[kGroupMax];
  int64_t M[kGroupMax], N[kGroupMax], K[kGroupMax];
  const void* A[kGroupMax];
  const void* W[kGroupMax];
  void* C[kGroupMax];
  int64_t lda[kGroupMax], ldw[kGroupMax], ldc[kGroupMax];
  int64_t sA[kGroupMax], sW[kGroupMax], sC[kGroupMax];
  float* sq_part;        // nullable: per-workgroup sum of squares of C (ea.sq_part)
  bool sq[kGroupMax];    // which problems' tiles count in it
};

template <typename TI, typename TO, bool MF16, bool TN = false>
__global__ __launch_bounds__(512, 2) void gemm256p_group_kernel(GemmGroup g) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * G2_STAGE];
  const int t = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  int p = 0;
  while (p + 1 < g.n && t >= g.tile_end[p]) ++p;
  const int local = t - (p ? g.tile_end[p - 1] : 0);
  const int b = local / g.tpb[p], lt = local - b * g.tpb[p];
  const int nx = g.ntn[p];
  EpiArgs ea{0, 0, g.alpha[p]};
  ea.sq_part = g.sq_part;
  ea.sq_on = g.sq[p];
  // an XCD runs ~32 consecutive ids at a time: grouped 4 M-tiles x 8 N-tiles
  // (tile_of), so its L2 holds 12 operand panels per K step, not 2 + 16
  int mt, nt;
  tile_of(lt, nx, (int)((g.M[p] + G2BM - 1) / G2BM), 4, mt, nt);
  gemm256p_body<TI, NR_EPI_NONE, TO, MF16, TN>(smem, (int64_t)mt * G2BM, (int64_t)nt * G2BN, g.M[p],
                                               g.N[p], g.K[p], (const TI*)g.A[p] + b * g.sA[p], g.lda[p],
                                               (const TI*)g.W[p] + b * g.sW[p], g.ldw[p], nullptr, nullptr, 0,
                                               (TO*)g.C[p] + b * g.sC[p], g.ldc[p], ea);
}

int gemm_group_dispatch(int dtype_in, int dtype_out, const GemmProblem* probs, int n, hipStream_t s, float* sq_part,
                        const bool* sq, int* n_tiles, int sq_cap) {
  NR_CHECK_ARG(dtype_in == NR_BF16 || dtype_in == NR_F32, "gemm_group: bad dtype_in %d", dtype_in);
  NR_CHECK_ARG(dtype_out == NR_F32 || dtype_out == NR_BF16, "gemm_group: bad dtype_out %d", dtype_out);
  NR_CHECK_ARG(n >= 0 && n <= kGroupMax, "gemm_group: n=%d outside [0, %d]", n, kGroupMax);
  GemmGroup g{};
  g.n = 0;
  int64_t tiles = 0;
  const int64_t bk = dtype_in == NR_F32 ? 32 : 64, e16 = dtype_in == NR_F32 ? 4 : 8;
  const int64_t vo = dtype_out == NR_F32 ? 4 : 8;
  for (int i = 0; i < n; ++i) {
    const GemmProblem& q = probs[i];
    NR_CHECK_ARG(q.M >= 0 && q.N > 0 && q.K > 0 && q.N % G2BN == 0 && q.K % bk == 0 && q.batch >= 0,
                 "gemm_group: problem %d bad shape M=%lld N=%lld K=%lld (need N %% 256, K %% 64 bf16 / 32 f32)", i,
                 (long long)q.M, (long long)q.N, (long long)q.K);
    if (q.M == 0 || q.batch == 0) continue;
    NR_CHECK_ARG(q.A && q.W && q.C, "gemm_group: problem %d null operand", i);
    NR_CHECK_ARG(q.lda >= q.K && q.ldw >= q.K && q.lda % e16 == 0 && q.ldw % e16 == 0 && q.ldc >= q.N &&
                     q.ldc % vo == 0 && ((uintptr_t)q.A & 15) == 0 && ((uintptr_t)q.W & 15) == 0 &&
                     ((uintptr_t)q.C & 15) == 0 && q.sA % e16 == 0 && q.sW % e16 == 0 && q.sC % vo == 0,
                 "gemm_group: problem %d operands must be 16-byte aligned with 16-byte row / batch strides", i);
    const int j = g.n++;
    g.M[j] = q.M; g.N[j] = q.N; g.K[j] = q.K;
    g.A[j] = q.A; g.W[j] = q.W; g.C[j] = q.C;
    g.lda[j] = q.lda; g.ldw[j] = q.ldw; g.ldc[j] = q.ldc;
    g.sA[j] = q.sA; g.sW[j] = q.sW; g.sC[j] = q.sC;
    g.alpha[j] = q.alpha;
    g.sq[j] = sq ? sq[i] : false;
    g.ntn[j] = (int)(q.N / G2BN);
    const int64_t tpb = ((q.M + G2BM - 1) / G2BM) * g.ntn[j];
    NR_CHECK_ARG(tpb <= 0x7fffffff, "gemm_group: too many tiles");
    g.tpb[j] = (int)tpb;
    tiles += tpb * q.batch;
    NR_CHECK_ARG(tiles <= 0x7fffffff, "gemm_group: too many tiles");
    g.tile_end[j] = (int)tiles;
  }
  if (n_tiles) *n_tiles = (int)tiles;
  if (g.n == 0) return NR_OK;
  NR_CHECK_ARG(!sq_part || tiles <= sq_cap, "gemm_group: %lld workgroups exceed the %d sum-of-squares slots",
               (long long)tiles, sq_cap);
  g.sq_part = sq_part;
  if (dtype_in == NR_F32 && dtype_out == NR_F32)
    hipLaunchKernelGGL((gemm256p_group_kernel<float, float, false>), dim3((unsigned)tiles), dim3(512), 0, s, g);
  else if (dtype_in == NR_F32)
    hipLaunchKernelGGL((gemm256p_group_kernel<float, __bf16, false>), dim3((unsigned)tiles), dim3(512), 0, s, g);
  else if (dtype_out == NR_F32)
    hipLaunchKernelGGL((gemm256p_group_kernel<__bf16, float, true>), dim3((unsigned)tiles), dim3(512), 0, s, g);
  else
    hipLaunchKernelGGL((gemm256p_group_kernel<__bf16, __bf16, true>), dim3((unsigned)tiles), dim3(512), 0, s, g);
  NR_CHECK_LAUNCH("gemm_group");
  return NR_OK;
}

// Grouped TN launch (gemm256p_body TN): problem i computes C = alpha A^T W with A
// [K][M] (row stride lda), W [K][N] (ldw), bf16, C [M][N] f32 or bf16 -- the
// weight-grad GEMMs dW = dOut^T X of the training steps on their row-major
// activations.  Batches (sA / sW / sC) give split-K slices: A + b sA is K-rows
// b kw.. of the same activation.  M, N multiples of 256, K of 64.
int gemm_group_tn_dispatch(int dtype_out, const GemmProblem* probs, int n, hipStream_t s, float* sq_part,
                           const bool* sq, int* n_tiles, int sq_cap) {
  NR_CHECK_ARG(dtype_out == NR_F32 || dtype_out == NR_BF16, "gemm_group_tn: bad dtype_out %d", dtype_out);
  NR_CHECK_ARG(n >= 0 && n <= kGroupMax, "gemm_group_tn: n=%d outside [0, %d]", n, kGroupMax);
  GemmGroup g{};
  int64_t tiles = 0;
  const int64_t vo = dtype_out == NR_F32 ? 4 : 8;
  for (int i = 0; i < n; ++i) {
    const GemmProblem& q = probs[i];
    NR_CHECK_ARG(q.M > 0 && q.N > 0 && q.K >= 0 && q.M % G2BM == 0 && q.N % G2BN == 0 && q.K % 64 == 0 &&
                     q.batch >= 0,
                 "gemm_group_tn: problem %d bad shape M=%lld N=%lld K=%lld (need M, N %% 256, K %% 64)", i,
                 (long long)q.M, (long long)q.N, (long long)q.K);
    if (q.K == 0 || q.batch == 0) continue;
    NR_CHECK_ARG(q.A && q.W && q.C, "gemm_group_tn: problem %d null operand", i);
    NR_CHECK_ARG(q.lda >= q.M && q.ldw >= q.N && q.lda % 8 == 0 && q.ldw % 8 == 0 && q.ldc >= q.N &&
                     q.ldc % vo == 0 && ((uintptr_t)q.A & 15) == 0 && ((uintptr_t)q.W & 15) == 0 &&
                     ((uintptr_t)q.C & 15) == 0 && q.sA % 8 == 0 && q.sW % 8 == 0 && q.sC % vo == 0,
                 "gemm_group_tn: problem %d operands must be 16-byte aligned with 16-byte row / batch strides", i);
    const int j = g.n++;
    g.M[j] = q.M; g.N[j] = q.N; g.K[j] = q.K;
    g.A[j] = q.A; g.W[j] = q.W; g.C[j] = q.C;
    g.lda[j] = q.lda; g.ldw[j] = q.ldw; g.ldc[j] = q.ldc;
    g.sA[j] = q.sA; g.sW[j] = q.sW; g.sC[j] = q.sC;
    g.alpha[j] = q.alpha;
    g.sq[j] = sq ? sq[i] : false;
    g.ntn[j] = (int)(q.N / G2BN);
    const int64_t tpb = (q.M / G2BM) * g.ntn[j];
    g.tpb[j] = (int)tpb;
    tiles += tpb * q.batch;
    NR_CHECK_ARG(tiles <= 0x7fffffff, "gemm_group_tn: too many tiles");
    g.tile_end[j] = (int)tiles;
  }
  if (n_tiles) *n_tiles = (int)tiles;
  if (g.n == 0) return NR_OK;
  NR_CHECK_ARG(!sq_part || tiles <= sq_cap, "gemm_group_tn: %lld workgroups exceed the %d sum-of-squares slots",
               (long long)tiles, sq_cap);
  g.sq_part = sq_part;
  if (dtype_out == NR_F32)
    hipLaunchKernelGGL((gemm256p_group_kernel<__bf16, float, true, true>), dim3((unsigned)tiles), dim3(512), 0, s, g);
  else
    hipLaunchKernelGGL((gemm256p_group_kernel<__bf16, __bf16, true, true>), dim3((unsigned)tiles), dim3(512), 0, s, g);
  NR_CHECK_LAUNCH("gemm_group_tn");
  return NR_OK;
}

// ---------------------------------------------------------------------------
// Persistent bf16 -> bf16 GEMM with a register-direct epilogue (the default
// for bf16 operands and bf16 output: every per-news transform GEMM and the
// bf16 encoder).  One 512-thread workgroup per CU walks its share of the
// 256x256 output tiles (8 XCD-contiguous ranges, the grouped tile order of
// tile_of), so a CU never idles between tiles waiting for a new workgroup.
// The main loop is gemm256p_body's 4-phase pipeline with the MFMA operands
// swapped (acc = W fragment x A fragment): the 16x16 accumulator of lane l
// then holds C[row l & 15][cols 4 (l >> 4) .. +3], which leave straight from
// registers (no LDS slab).
// One operand stream across tiles: the K steps of a workgroup's consecutive
// tiles form one sequence (stage = parity of the position in it), so the last
// two K steps of a tile prefetch the next tile's first two steps and bias
// slice exactly as they would K steps of their own.  The epilogue then runs with the
// next tile's operands already resident: no prologue and no operand wait at a
// tile boundary.  The two wave groups (skewed by one barrier in the main loop)
// are realigned for the epilogue, so both groups' epilogues run at once (one
// wave of each per SIMD), and re-skewed after it (measured against keeping
// the skew across the boundary, which serialises the two epilogues: 2-8 %
// faster, 17 % on softmax64; profiles/round2/gemm_persist).  Operand DMAs go
// through buffer descriptors: the per-lane 32-bit offsets are fixed per tile,
// the K offset rides in an SGPR (host: every operand < 4 GiB).
__device__ __forceinline__ uint4 swap_pair16(uint2 a, uint2 b) {
  // Row-segment of two adjacent 16-column tiles (a = tile 0, b = tile 1) of a
  // swapped-operand 16x16 accumulator: lane (row l & 15, q = l >> 4) holds
  // columns 4q..4q+3 of each tile as packed bf16.  One v_permlane16_swap per
  // dword (lanes 16-31 / 48-63 of `a` <-> lanes 0-15 / 32-47 of `b`) leaves
  // lanes with even q holding tile 0, columns 8 (q / 2) .. +7, and lanes with
  // odd q tile 1, columns 8 (q / 2) .. +7: 16 contiguous bytes per lane at
  // column 16 (q & 1) + 8 (q >> 1) (guide T21, here with the 16-lane swap).
  // The swap pairs lanes of one row, and is its own inverse.
  const auto sx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto sy = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  return uint4{sx[0], sy[0], sx[1], sy[1]};
}

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ uint32_t relu_bf16x2(uint32_t v) {  // v_pk_max_i16 with 0
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2, v), i16x2{0, 0}));
}

// s_waitcnt immediates waiting on vmcnt only (gfx9 encoding: vmcnt [3:0] and
// [15:14], expcnt [6:4] = 7, lgkmcnt [11:8] = 15).  Issued through the builtin,
// not inline asm, so the compiler's own wait insertion sees them: it then knows
// the older stores have retired and keeps its waits for the epilogue's
// residual loads counted instead of vmcnt(0).
constexpr unsigned kVmcnt0 = 0x0F70, kVmcnt4 = 0x0F74, kVmcnt8 = 0x0F78, kVmcnt6 = 0x0F76, kVmcnt9 = 0x0F79;  // lgkmcnt/expcnt left at max

// LNF (LayerNorm folded into the epilogue): per tile, every wave's (u, c)
// column slices (2 x 256 B) and the tile's 256 row stats (2 KiB), in two
// slots (tile parity): tile t + 1's slot is filled by the DMAs that prefetch
// its first K step while tile t's epilogue still reads slot t.
constexpr int kLnSlot = 8 * 512 + 256 * 8;

// CS (column sums, the training steps' bias gradients): every wave also writes
// the f32 column sums of its 128 output rows (the epilogue values before the
// bf16 rounding, rows past M excluded) to ea.colsum row (m0 + 128 wm) / 128,
// so db = the sum of those ceil(M / 128) rows, with no re-read of the output.
template <int EPI, bool LNF = false, bool CS = false>
__global__ __launch_bounds__(512, 2) void gemm256t_kernel(int64_t M, int64_t N, int64_t K,
                                                          const __bf16* __restrict__ A, int64_t lda,
                                                          const __bf16* __restrict__ W, int64_t ldw,
                                                          const float* __restrict__ bias, const __bf16* R,
                                                          int64_t ldr, __bf16* C, int64_t ldc, EpiArgs ea,
                                                          int ntn, int ntm, int n_tiles, int n_half) {
  constexpr int BK = 64;
  // operand stages + one 256-B bias slice per wave (LDS-DMA'd with the tile's step 0)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * G2_STAGE + 8 * 256 + (LNF ? 2 * kLnSlot : 0)];
  // wave-derived values are scalars (readfirstlane): VGPRs are the kernel's limit
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int wmu = wm;
  const int nk = (int)(K / BK);  // >= 2 (host)

  // tile schedule: XCD group x = blockIdx % 8 owns a contiguous range of tile
  // ids; its ~32 workgroups run consecutive ids, which tile_of groups into
  // 4 M-tiles x 8 N-tiles sharing A and W panels in that XCD's L2
  const int G = (int)gridDim.x;
  int t, t_end, t_step;
  if (G % 8 == 0) {
    const int x = (int)blockIdx.x & 7, li = (int)blockIdx.x >> 3;
    const int qq = n_tiles >> 3, rr = n_tiles & 7;
    const int lo = x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq;
    t = lo + li;
    t_end = lo + qq + (x < rr ? 1 : 0);
    t_step = G >> 3;
  } else {
    t = (int)blockIdx.x;
    t_end = n_tiles;
    t_step = G;
  }
  // Units: full tiles 0 .. n_tiles - 1 (whole rounds of the grid), then the
  // tiles of the last partial round cut into 128-row halves, unit n_tiles + h
  // = half h & 1 of tile n_tiles + h / 2, one per workgroup h < n_half
  // (host: only when they fit one round).  A half is computed by wave group
  // 0 alone (rows mb .. mb + 127) with the same per-element K chain and
  // epilogue as a full tile, so every row's bits are independent of the cut;
  // group 1 keeps its barriers and DMA pieces and skips reads, MFMAs and
  // stores.  The tail round then takes a half tile's time instead of a
  // tile's (at M = 72,023, N = 1024: 4 rounds + 208 halves, not 5 rounds).
  const int hb = (int)blockIdx.x < n_half ? n_tiles + (int)blockIdx.x : -1;
  int u = t < t_end ? t : hb;
  if (u < 0) return;  // workgroup-uniform
  auto next_unit = [&](int cur) { return cur < n_tiles ? (cur + t_step < t_end ? cur + t_step : hb) : -1; };
  auto tile_base = [&](int unit, uint32_t& mb, uint32_t& nb) {
    int mt, nt, tile = unit;
    uint32_t off = 0;
    if (unit >= n_tiles) {
      tile = n_tiles + ((unit - n_tiles) >> 1);
      off = (uint32_t)((unit - n_tiles) & 1) * (G2BM / 2);
    }
    tile_of(tile, ntn, ntm, ea.group_m, mt, nt);
    mb = (uint32_t)mt * G2BM + off;
    nb = (uint32_t)nt * G2BN;
  };

  // buffer descriptors over A, W and the bias, built from readfirstlane'd
  // kernel arguments so the compiler can prove them wave-uniform (T20: else
  // every buffer op gets a waterfall loop)
  auto rsrc = [](const void* p, int64_t bytes) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const int n = __builtin_amdgcn_readfirstlane((int)(bytes > 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)bytes));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
  };
  // per-tile descriptors: A from the unit's first row (its range = the rows
  // left, so rows past M fail the range check on the VGPR offset alone and
  // read zeros), W from the tile's first column; the per-lane offsets below
  // are then the same for every tile
  __amdgpu_buffer_rsrc_t rA, rW;
  // (a half unit may start past M: no records then)
  auto set_tileA = [&](uint32_t mb) { rA = rsrc(A + (int64_t)mb * lda, max(M - (int64_t)mb, (int64_t)0) * lda * 2); };
  auto set_tileB = [&](uint32_t nb) { rW = rsrc(W + (int64_t)nb * ldw, (N - (int64_t)nb) * ldw * 2); };
  // DMA units are the quarters the phases finish reading: A unit q = rows
  // 64 q .. +63 of both wave-group halves (lane l of wave w: row
  // 128 (w >> 2) + 64 q + 16 (w & 3) + 8 j + l / 8), B unit q = rows 32 q .. +31
  // of all four wn slices (row 64 (w >> 1) + 32 q + 16 (w & 1) + 8 j + l / 8);
  // 16-B chunk (l & 7) ^ ((row >> 1) & 7) of the LDS image (T2 swizzle on the
  // source).  Per-lane offsets relative to the tile's descriptors, fixed for
  // the whole launch: A per (unit, j) (a row past M must fail the range check
  // on its own VGPR offset), B per j with the unit's 32 rows in the scalar
  // offset (W rows are always in range).  Rows past M are never stored.
  const int qa = (wave >> 2) * 128 + (wave & 3) * 16, qb = (wave >> 1) * 64 + (wave & 1) * 16;
  const uint32_t ldab = (uint32_t)lda * 2, ldwb = (uint32_t)ldw * 2, mlast = (uint32_t)(M - 1);
  auto chunk = [&](int j) { return (uint32_t)(((lane & 7) ^ ((4 * j + (lane >> 4)) & 7)) * 16); };
  uint32_t oA[2][2], oB[2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) oA[h][j] = (uint32_t)(qa + 64 * h + 8 * j + (lane >> 3)) * ldab + chunk(j);
#pragma unroll
  for (int j = 0; j < 2; ++j) oB[j] = (uint32_t)(qb + 8 * j + (lane >> 3)) * ldwb + chunk(j);
  auto dmaA = [&](int h, int stage, int kt) {
    unsigned char* sa = smem + stage * G2_STAGE + (qa + 64 * h) * 128;
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)kt * (BK * 2));
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(sa + 8 * j * 128), 16, oA[h][j], so, 0, 0);
  };
  auto dmaB = [&](int h, int stage, int kt) {
    unsigned char* sb = smem + stage * G2_STAGE + G2BM * 128 + (qb + 32 * h) * 128;
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)kt * (BK * 2) + (uint32_t)h * 32u * ldwb);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(sb + 8 * j * 128), 16, oB[j], so, 0, 0);
  };
  unsigned char* bias_lds = smem + 2 * G2_STAGE + wave * 256;  // this wave's 64 bias floats
  // (a buffer op like the operands: a global_load_lds here would be a FLAT
  // instruction, whose pending LDS write makes the compiler wait vmcnt(0))
  const __amdgpu_buffer_rsrc_t rBias = rsrc(bias, N * 4);
  auto dma_bias = [&](uint32_t nb) {
    if (bias)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rBias, (lds_void*)bias_lds, 4, (nb + (uint32_t)(wn * 64 + lane)) * 4, 0,
                                               0, 0);
  };
  // LNF: 3 single-dword DMAs per wave (u slice, c slice, 32 of the tile's row stats)
  unsigned char* ln_lds = smem + 2 * G2_STAGE + 8 * 256;
  const __amdgpu_buffer_rsrc_t rUC = rsrc(ea.ln_uc, LNF ? 2 * N * 4 : 0);
  const __amdgpu_buffer_rsrc_t rST = rsrc(ea.ln_stats, LNF ? M * 8 : 0);
  auto dma_ln = [&](int slot, uint32_t mb, uint32_t nb) {
    if constexpr (LNF) {
      unsigned char* base = ln_lds + slot * kLnSlot;
      const uint32_t cu = (nb + (uint32_t)(wn * 64 + lane)) * 4;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rUC, (lds_void*)(base + wave * 512), 4, cu, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rUC, (lds_void*)(base + wave * 512 + 256), 4, cu + (uint32_t)N * 4, 0, 0,
                                               0);
      const uint32_t row = min(mb + (uint32_t)(32 * wave + (lane >> 1)), mlast);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rST, (lds_void*)(base + 8 * 512 + wave * 256), 4,
                                               row * 8 + (uint32_t)(lane & 1) * 4, 0, 0, 0);
    }
  };
  int lslot = 0;  // LNF slot of the current tile

  // fragment reads (16x16x32 operand map: row lane & 15, k chunk 4 f + lane / 16)
  const int c16 = lane & 15, q4 = lane >> 4;
  const int sw = (c16 >> 1) & 7;
  const int abase = (wm * 128 + c16) * 128;
  const int bbase = G2BM * 128 + (wn * 64 + c16) * 128;
  const int cf0 = ((0 + q4) ^ sw) << 4, cf1 = ((4 + q4) ^ sw) << 4;
  typedef f32x4 frag_t;
  frag_t fa[4][2], fbx[2][2], fby[2][2];  // [row tile][k half]; B fragments in two alternating sets
  f32x4 acc[8][4];
  auto readA = [&](int stage, int qm) {
    const unsigned char* sp = smem + stage * G2_STAGE + abase + qm * 4 * 2048;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i][0] = *reinterpret_cast<const frag_t*>(sp + i * 2048 + cf0);
      fa[i][1] = *reinterpret_cast<const frag_t*>(sp + i * 2048 + cf1);
    }
  };
  auto readB = [&](int stage, int qn, frag_t (&fb)[2][2]) {
    const unsigned char* sp = smem + stage * G2_STAGE + bbase + qn * 2 * 2048;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fb[j][0] = *reinterpret_cast<const frag_t*>(sp + j * 2048 + cf0);
      fb[j][1] = *reinterpret_cast<const frag_t*>(sp + j * 2048 + cf1);
    }
  };
  // swapped operands: D[n][m] = sum_k W[n][k] A[m][k] = C[m][n]
  auto mma = [&](int qm, int qn, const frag_t (&fb)[2][2]) {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 * qm + i][2 * qn + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, fb[j][f]), __builtin_bit_cast(bf16x8, fa[i][f]), acc[4 * qm + i][2 * qn + j],
              0, 0, 0);
  };
#define NR_PHASE_SYNC_MMA(QM, NI, FB)                   \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
  __builtin_amdgcn_sched_barrier(0);                   \
  __builtin_amdgcn_s_barrier();                        \
  __builtin_amdgcn_s_setprio(1);                       \
  if constexpr (!IDLE) mma(QM, NI, FB);               \
  __builtin_amdgcn_s_setprio(0);                       \
  __builtin_amdgcn_s_barrier();
  // K step kt of the current tile (stage st).  Step kt + 2 is prefetched into
  // this stage, each quarter at least one phase after its last read (both
  // wave groups' reads of phase p retire before the barrier instance the
  // leading group passes to enter phase p + 1), two 1-KiB pieces per wave in
  // every phase: A0 in P2 (read in P1), B0 in P3 (read in the previous step's
  // P4), B1 in P4 (read in P2), and A1 (read in P3) in the NEXT step's P1 --
  // this tile's step, or past its end the next tile's steps 0 and 1 (with the
  // next tile's bias slice ahead of step 0).  P4 then waits for step kt + 1
  // (its A1 issued in this step's P1) with 6 pieces of step kt + 2 in flight.
  // Fragment reads per phase 8 / 4 / 8 / 4 (round 4; was 12 / 4 / 8 / 0): P4
  // reads step kt + 1's B0 into the B set P3 has finished with, so the two B
  // sets swap roles every step (B0 in fbx on even steps, in fby on odd ones);
  // P3 waits (vmcnt 8) for step kt + 1's B0, issued in step kt - 1's P3, so
  // that P4 reads it one phase after the wait.  A tile's step-0 B0 is read at
  // the tile top (retired by the previous tile's last P4 wait, or the
  // prologue's, and a barrier since) and its last step reads none in P4, so no
  // fragments live across the epilogue.
  bool a1p = false;  // the previous step's A1 refill (stage st ^ 1, step a1k), issued in this step's P1
  int a1k = 0;
  // fb0: this step's B0 (rows qn = 0); fb1: its B1, then step kt + 1's B0
  auto kstep = [&](auto idle, int kt, int st, bool more, uint32_t nm0, uint32_t nn0, frag_t(&fb0)[2][2],
                   frag_t(&fb1)[2][2]) __attribute__((always_inline)) {
    constexpr bool IDLE = decltype(idle)::value;
    const bool pf = kt + 2 < nk || more;
    const int kf = kt + 2 < nk ? kt + 2 : kt + 2 - nk;
    if constexpr (!IDLE) readA(st, 0);
    if (a1p) dmaA(1, st ^ 1, a1k);
    NR_PHASE_SYNC_MMA(0, 0, fb0)
    if constexpr (!IDLE) readB(st, 1, fb1);
    if (pf) {
      if (kt + 2 == nk) {
        set_tileA(nm0);
        set_tileB(nn0);
        dma_bias(nn0);
      }
      dmaA(0, st, kf);
    }
    NR_PHASE_SYNC_MMA(0, 1, fb1)
    if constexpr (!IDLE) readA(st, 1);
    if (pf) dmaB(0, st, kf);
    // step kt + 1's B0 landed (read in P4): issued after it are its B1 and A1
    // and, when pf, step kt + 2's A0 and B0 (2 instructions each; a bias or LN
    // DMA among them only makes the wait stricter)
    if (pf)
      __builtin_amdgcn_s_waitcnt(kVmcnt8);
    else
      __builtin_amdgcn_s_waitcnt(kVmcnt4);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if constexpr (!IDLE) {
      if (kt + 1 < nk) readB(st ^ 1, 0, fb1);
    }
    if (pf) {
      dmaB(1, st, kf);
      if (LNF && kt + 2 == nk) {
        dma_ln(lslot ^ 1, nm0, nn0);
        __builtin_amdgcn_s_waitcnt(kVmcnt9);
      } else {
        __builtin_amdgcn_s_waitcnt(kVmcnt6);  // step kt + 1 landed (incl. its A1 from P1); 6 of kt + 2 fly
      }
    } else {
      __builtin_amdgcn_s_waitcnt(kVmcnt0);
    }
    a1p = pf;
    a1k = kf;
    __builtin_amdgcn_sched_barrier(0);  // the B0 reads stay ahead of the MFMA cluster (not waited for: P4's MFMAs do not use them)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
    if constexpr (!IDLE) mma(1, 0, fb0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };
  // a tile's K loop: steps in (even, odd) pairs (nk even, host), B0 in fbx on
  // even steps; every tile starts on stage 0
  auto kloop = [&](auto idle, bool more, uint32_t nm0, uint32_t nn0) __attribute__((always_inline)) {
    for (int kt = 0; kt < nk; kt += 2) {
      kstep(idle, kt, 0, more, nm0, nn0, fbx, fby);
      kstep(idle, kt + 1, 1, more, nm0, nn0, fby, fbx);
    }
  };

  uint32_t m0, n0;
  tile_base(u, m0, n0);
  set_tileA(m0);
  set_tileB(n0);
  // first tile: LN slices, bias slice + steps 0 and 1 (stages 0 and 1)
  dma_ln(0, m0, n0);
  dma_bias(n0);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    dmaB(0, k, k);
    dmaB(1, k, k);
    dmaA(0, k, k);
    dmaA(1, k, k);
  }
  __builtin_amdgcn_s_waitcnt(kVmcnt8);
  __builtin_amdgcn_s_barrier();
  if (wmu == 1) __builtin_amdgcn_s_barrier();  // skew the wave groups by one barrier
  while (true) {
    const int tn = next_unit(u);
    const bool more = tn >= 0;
    if (u >= n_tiles && wmu == 1) break;  // group 1 of a half unit: below
    uint32_t nm0 = 0, nn0 = 0;
    if (more) tile_base(tn, nm0, nn0);
    // the accumulators start at the bias (acc = bias + A.W^T); this wave's
    // columns wn*64 + 16 ni + 4 q4 .. +3
    if constexpr (LNF) {
      // LNF: acc starts at -mean(row) u(col), so the epilogue is one fma per
      // element, rstd acc + c (the tile's LN slot landed with its step 0)
      const unsigned char* ls = ln_lds + lslot * kLnSlot;
      f32x4 u4[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) u4[ni] = *reinterpret_cast<const f32x4*>(ls + wave * 512 + (16 * ni + 4 * q4) * 4);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const float nmean = -*reinterpret_cast<const float*>(ls + 8 * 512 + (wm * 128 + c16 + 16 * mi) * 8);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = nmean * u4[ni];
      }
    } else {
      f32x4 b4[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        b4[ni] = bias ? *reinterpret_cast<const f32x4*>(bias_lds + (16 * ni + 4 * q4) * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = b4[ni];
    }
    readB(0, 0, fbx);  // step 0's B0
    kloop(std::false_type{}, more, nm0, nn0);

    if (wmu == 0) __builtin_amdgcn_s_barrier();  // realign: group 1 has finished its last MFMA phase
    {
    // ---------------- epilogue of tile (m0, n0) ----------------
    // The next tile's first stage is resident or in flight; nothing here
    // touches LDS or waits on the operand DMAs.  Rows past M are clamped to
    // M - 1 (their A rows were clamped by the DMA too) for every load, but do
    // not store: with an in-place residual (R == C, the latent ff2) another
    // wave group's duplicate store of row M - 1 could land before this
    // group's residual load of it and add the residual twice.
    const int64_t row0 = (int64_t)m0 + wm * 128 + c16;  // + 16 mi
    const int64_t col0 = (int64_t)n0 + wn * 64;          // this wave's 64 columns
    const int qo = 16 * (q4 & 1) + 8 * (q4 >> 1);        // lane's 8 columns after swap_pair16
    // LNF: this lane's 16 columns' (u, c) and the tile's row stats (slot lslot)
    // (re-read from LDS per row group: 32 VGPRs held across the epilogue spilled)
    const unsigned char* ln_st = ln_lds + lslot * kLnSlot + 8 * 512;
    const unsigned char* ln_uc = ln_lds + lslot * kLnSlot + wave * 512;
    // residual (softmax backward: the softmax output P) in the store layout (16
    // B per lane): a window of 4 row groups in flight, row group mi + 4 loaded
    // into mi's slot once mi is stored (all 8 up front held 64 VGPRs beside the
    // accumulators and spilled)
    uint4 rq[4][2];
    auto load_r = [&](int mi) {
      const int64_t row = min(row0 + 16 * mi, M - 1);
#pragma unroll
      for (int p = 0; p < 2; ++p) rq[mi & 3][p] = *reinterpret_cast<const uint4*>(R + row * ldr + col0 + 32 * p + qo);
      __builtin_amdgcn_sched_barrier(0);  // issue order = use order: counted waits, not vmcnt(0)
    };
    constexpr bool kRes = EPI == NR_EPI_RESADD || EPI == NR_EPI_SOFTMAX64_BWD || EPI == NR_EPI_DRELU;
    if constexpr (kRes) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) load_r(mi);
    }
    f32x4 cs[4];  // CS: this lane's column partial sums (columns 16 ni + 4 q4 .. +3)
    if constexpr (CS) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) cs[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int64_t row = min(row0 + 16 * mi, M - 1);
      const bool live = row0 + 16 * mi < M;  // clamped duplicates of row M - 1 never store
      if constexpr (LNF) {
        // LN(a) . w = rstd (a . (w o gamma) - mean u) + c   (row stats of the A row;
        // acc started at -mean u)
        asm volatile("" ::: "memory");  // no CSE of the c reads across row groups
        const float rstd = *reinterpret_cast<const float*>(ln_st + (wm * 128 + c16 + 16 * mi) * 8 + 4);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const f32x4 lc = *reinterpret_cast<const f32x4*>(ln_uc + 256 + (16 * ni + 4 * q4) * 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[mi][ni][r] = fmaf(rstd, acc[mi][ni][r], lc[r]);
        }
      }
      if constexpr (EPI == NR_EPI_GEGLU) {
        // W rows interleaved in 32-row (a, g) blocks: ni 0, 1 = a, ni 2, 3 = g
        uint2 pk[2];
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          f32x2v g0 = (f32x2v){acc[mi][ni + 2][0], acc[mi][ni + 2][1]};
          f32x2v g1 = (f32x2v){acc[mi][ni + 2][2], acc[mi][ni + 2][3]};
          gelu_erf2x2(g0, g1);
          const f32x2v o0 = (f32x2v){acc[mi][ni][0], acc[mi][ni][1]} * g0;
          const f32x2v o1 = (f32x2v){acc[mi][ni][2], acc[mi][ni][3]} * g1;
          pk[ni] = uint2{pack_bf16x2(o0.x, o0.y), pack_bf16x2(o1.x, o1.y)};
        }
        const uint4 v = swap_pair16(pk[0], pk[1]);
        if (live) *reinterpret_cast<uint4*>(C + row * ldc + col0 / 2 + qo) = v;
        __builtin_amdgcn_sched_barrier(0);  // one row group at a time: bounds the erf temporaries' live ranges
      } else {
        if constexpr (EPI == NR_EPI_RESADD) {
          // the residual to the accumulator layout by the same (involutive) swap
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const uint4 s = swap_pair16(uint2{rq[mi & 3][p].x, rq[mi & 3][p].y}, uint2{rq[mi & 3][p].z, rq[mi & 3][p].w});
            const uint32_t w[2][2] = {{s.x, s.y}, {s.z, s.w}};  // tile 2p, tile 2p + 1
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const uint32_t u = w[h][r >> 1];
                acc[mi][2 * p + h][r] += (r & 1) ? bf16_hi(u) : bf16_lo(u);
              }
          }
        }
        if constexpr (EPI == NR_EPI_DRELU) {
          // relu / dropout backward: dZ = dY * (y > 0 ? 1 / (1 - p) : 0), y = the
          // forward output (R) in the accumulator layout by the same swap
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const uint4 s = swap_pair16(uint2{rq[mi & 3][p].x, rq[mi & 3][p].y}, uint2{rq[mi & 3][p].z, rq[mi & 3][p].w});
            const uint32_t w[2][2] = {{s.x, s.y}, {s.z, s.w}};
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const uint32_t u = w[h][r >> 1];
                const float y = (r & 1) ? bf16_hi(u) : bf16_lo(u);
                acc[mi][2 * p + h][r] = y > 0.f ? acc[mi][2 * p + h][r] * ea.scale : 0.f;
              }
          }
        }
        float v[4][4];
        if constexpr (EPI == NR_EPI_SOFTMAX64_BWD) {
          // dS = P (dP - sum_group P dP): acc = dP, P from R in the accumulator layout;
          // the wave's 64 columns are one softmax group (lanes l, l ^ 16, l ^ 32, l ^ 48)
          float pv[4][4];
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const uint4 sw = swap_pair16(uint2{rq[mi & 3][p].x, rq[mi & 3][p].y}, uint2{rq[mi & 3][p].z, rq[mi & 3][p].w});
            const uint32_t w[2][2] = {{sw.x, sw.y}, {sw.z, sw.w}};
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const uint32_t u = w[h][r >> 1];
                pv[2 * p + h][r] = (r & 1) ? bf16_hi(u) : bf16_lo(u);
              }
          }
          float dot = 0.f;
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) dot = fmaf(pv[ni][r], acc[mi][ni][r], dot);
          dot += __shfl_xor(dot, 16, 64);
          dot += __shfl_xor(dot, 32, 64);
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[mi][ni][r] = pv[ni][r] * (acc[mi][ni][r] - dot);
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          // the lane's 4 consecutive columns col0 + 16 ni + 4 q4 .. +3 are one group
          // of the dropout stream: one hash for the four
          uint64_t dh = 0;
          if constexpr (EPI == NR_EPI_RELU_DROPOUT) dh = drop_hash4(ea.seed, (uint64_t)(row * N + col0 + 16 * ni + 4 * q4) >> 2);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = acc[mi][ni][r];
            if constexpr (EPI == NR_EPI_RELU_DROPOUT) x = drop_field(dh, r, ea.thr) ? 0.f : fmaxf(x, 0.f) * ea.scale;
            if constexpr (EPI == NR_EPI_EXP) x = epi_exp(x);
            v[ni][r] = x;
          }
        }
        if constexpr (EPI == NR_EPI_GELU) {
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) {
            f32x2v g0 = (f32x2v){v[ni][0], v[ni][1]}, g1 = (f32x2v){v[ni][2], v[ni][3]};
            gelu_erf2x2(g0, g1);
            v[ni][0] = g0.x;
            v[ni][1] = g0.y;
            v[ni][2] = g1.x;
            v[ni][3] = g1.y;
          }
        }
        if constexpr (EPI == NR_EPI_SOFTMAX64) {
          // the wave's 64 columns are one softmax group; row (l & 15)'s values
          // sit in lanes l, l ^ 16, l ^ 32, l ^ 48 (4 x 4 each)
          float mx = v[0][0];
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) mx = fmaxf(mx, v[ni][r]);
          mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
          mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
          float sum = 0.f;
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[ni][r] = epi_exp(v[ni][r] - mx);
              sum += v[ni][r];
            }
          sum += __shfl_xor(sum, 16, 64);
          sum += __shfl_xor(sum, 32, 64);
          const float inv = 1.0f / sum;
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[ni][r] *= inv;
        }
        if constexpr (CS) {
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) cs[ni][r] += live ? v[ni][r] : 0.f;
        }
        uint2 pk[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          pk[ni] = uint2{pack_bf16x2(v[ni][0], v[ni][1]), pack_bf16x2(v[ni][2], v[ni][3])};
          // ReLU on the packed bf16: a set sign bit is a negative int16, so the
          // signed max with 0 zeroes exactly the negative values (and -0)
          if constexpr (EPI == NR_EPI_RELU) pk[ni] = uint2{relu_bf16x2(pk[ni].x), relu_bf16x2(pk[ni].y)};
        }
        const uint4 s0 = swap_pair16(pk[0], pk[1]), s1 = swap_pair16(pk[2], pk[3]);
        __bf16* dst = C + row * ldc + col0 + qo;
        if (live) {
          *reinterpret_cast<uint4*>(dst) = s0;
          *reinterpret_cast<uint4*>(dst + 32) = s1;
        }
        if constexpr (kRes) {
          __builtin_amdgcn_sched_barrier(0);  // row groups in load order
          if (mi + 4 < 8) load_r(mi + 4);
        }
      }
    }
    if constexpr (CS) {
      // sum over the 16 row lanes (c16) of each column; lane c16 < 4 stores columns 16 c16 + 4 q4 .. +3
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = cs[ni][r];
          x += __shfl_xor(x, 1, 64);
          x += __shfl_xor(x, 2, 64);
          x += __shfl_xor(x, 4, 64);
          x += __shfl_xor(x, 8, 64);
          cs[ni][r] = x;
        }
      // (a 128-row block wholly past M has no column-sum row: ceil(M / 128) rows)
      if (c16 < 4 && (int64_t)m0 + wm * 128 < M) {
        const f32x4 o = c16 == 0 ? cs[0] : c16 == 1 ? cs[1] : c16 == 2 ? cs[2] : cs[3];
        const int64_t prow = ((int64_t)m0 + wm * 128) >> 7;
        *reinterpret_cast<f32x4*>(ea.colsum + prow * N + col0 + 16 * c16 + 4 * q4) = o;
      }
    }
    }
    if (!more) break;
    if (wmu == 1) __builtin_amdgcn_s_barrier();  // re-skew
    lslot ^= 1;
    u = tn;
    m0 = nm0;
    n0 = nn0;
  }
  if (u >= n_tiles && wmu == 1) {  // the half unit's K loop for group 1 (its last unit: nothing to prefetch)
    kloop(std::true_type{}, false, 0u, 0u);
  }
#undef NR_PHASE_SYNC_MMA
}

// Workgroups of a persistent GEMM launch: the device's CU count rounded down
// to a multiple of the 8 XCDs, unless the caller has set a budget for a
// CU-masked stream (nr_set_persistent_workgroups).
// Process-wide knobs are atomics: the C-ABI is callable from several host
// threads at once (one stream each).
static std::atomic<int> g_persist_wgs{0};

extern "C" int nr_set_persistent_workgroups(int n) {
  if (n < 0 || n % 8) {
    set_error("nr_set_persistent_workgroups: n=%d must be 0 or a positive multiple of 8", n);
    return NR_ERR_INVALID;
  }
  g_persist_wgs.store(n);
  return NR_OK;
}

extern "C" int nr_persistent_workgroups(void) { return g_persist_wgs.load(); }

static int num_cus() {
  if (const int b = g_persist_wgs.load()) return b;
  static std::atomic<int> n_cu{0};  // racing first calls store the same value
  int c = n_cu.load(std::memory_order_relaxed);
  if (!c) {
    int dev = 0;
    hipDeviceProp_t prop;
    const int n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
                      ? prop.multiProcessorCount : 256;
    c = n >= 8 ? n / 8 * 8 : 8;
    n_cu.store(c, std::memory_order_relaxed);
  }
  return c;
}

// Half-tile tail (gemm256t_kernel's units): on unless a tuning caller turned it off.
static std::atomic<int> g_half_tail{1};

extern "C" int nr_set_gemm_half_tail(int on) {
  g_half_tail.store(on ? 1 : 0);
  return NR_OK;
}

// Persistent grid over `tiles` output tiles: *nt full tiles (whole rounds)
// and *nh half units (the last partial round's tiles cut in two, when they
// fit one round); returns the workgroup count.
static int persistent_schedule(int64_t tiles, int* nt, int* nh) {
  const int ncu = num_cus();
  const int rem = (int)(tiles % ncu);
  const bool split = g_half_tail.load() && rem > 0 && 2 * rem <= ncu;
  *nt = (int)tiles - (split ? rem : 0);
  *nh = split ? 2 * rem : 0;
  return *nt >= ncu ? ncu : (*nt > *nh ? *nt : *nh);
}

// The persistent kernel's operand stream needs an even number (>= 2) of
// 64-deep K steps per tile (its K loop runs them in pairs, the B fragment sets
// swapping roles) and addresses A and W through 32-bit buffer offsets.
static bool persistent_ok(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldw) {
  constexpr int64_t kMax = 0xFFFFFFFFll;
  return K >= 128 && K % 128 == 0 && M * lda * 2 <= kMax && N * ldw * 2 <= kMax;
}

static int launch_gemm256_t(int epi, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* W,
                            int64_t ldw, const float* bias, const void* R, int64_t ldr, void* C, int64_t ldc,
                            const EpiArgs& ea, hipStream_t s) {
  const int ntn = (int)(N / G2BN);
  const int64_t ntm = (M + G2BM - 1) / G2BM;
  const int64_t tiles = ntm * ntn;
  if (tiles > (1ll << 30)) {
    set_error("nr_gemm: too many tiles");
    return NR_ERR_UNSUPPORTED;
  }
  int nt, nh;
  const dim3 grid((unsigned)persistent_schedule(tiles, &nt, &nh));
  const __bf16* a = (const __bf16*)A;
  const __bf16* w = (const __bf16*)W;
  const __bf16* r = (const __bf16*)R;
  __bf16* c = (__bf16*)C;
#define NR_T(E) hipLaunchKernelGGL((gemm256t_kernel<E>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea, ntn, (int)ntm, nt, nh)
#define NR_TC(E) hipLaunchKernelGGL((gemm256t_kernel<E, false, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea, ntn, (int)ntm, nt, nh)
  if (ea.colsum) {
    switch (epi) {
      case NR_EPI_NONE: NR_TC(NR_EPI_NONE); break;
      case NR_EPI_RESADD: NR_TC(NR_EPI_RESADD); break;
      case NR_EPI_DRELU: NR_TC(NR_EPI_DRELU); break;
      default: set_error("nr_gemm: column sums with epilogue %d unsupported", epi); return NR_ERR_INVALID;
    }
    NR_CHECK_LAUNCH("nr_gemm");
    return NR_OK;
  }
#undef NR_TC
  switch (epi) {
    case NR_EPI_DRELU: NR_T(NR_EPI_DRELU); break;
    case NR_EPI_NONE: NR_T(NR_EPI_NONE); break;
    case NR_EPI_RELU: NR_T(NR_EPI_RELU); break;
    case NR_EPI_EXP: NR_T(NR_EPI_EXP); break;
    case NR_EPI_GEGLU: NR_T(NR_EPI_GEGLU); break;
    case NR_EPI_RESADD: NR_T(NR_EPI_RESADD); break;
    case NR_EPI_GELU: NR_T(NR_EPI_GELU); break;
    case NR_EPI_RELU_DROPOUT: NR_T(NR_EPI_RELU_DROPOUT); break;
    case NR_EPI_SOFTMAX64: NR_T(NR_EPI_SOFTMAX64); break;
    case NR_EPI_SOFTMAX64_BWD: NR_T(NR_EPI_SOFTMAX64_BWD); break;
    default: set_error("nr_gemm: bad epilogue %d", epi); return NR_ERR_INVALID;
  }
#undef NR_T
  NR_CHECK_LAUNCH("nr_gemm");
  return NR_OK;
}

template <typename TI, typename TO>
static int launch_gemm256_p(int epi, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                          const void* W, int64_t ldw, const float* bias, const void* R, int64_t ldr,
                          void* C, int64_t ldc, const EpiArgs& ea, hipStream_t s) {
  dim3 grid((unsigned)(N / G2BN), (unsigned)((M + G2BM - 1) / G2BM));
  const TI* a = (const TI*)A;
  const TI* w = (const TI*)W;
  const TO* r = (const TO*)R;
  TO* c = (TO*)C;
  switch (epi) {
    case NR_EPI_NONE: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_NONE, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RELU: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_RELU, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_EXP: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_EXP, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_GEGLU: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_GEGLU, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RESADD: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_RESADD, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_GELU: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_GELU, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RELU_DROPOUT: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_RELU_DROPOUT, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_DRELU: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_DRELU, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_SOFTMAX64: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_SOFTMAX64, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    default: set_error("nr_gemm: bad epilogue %d", epi); return NR_ERR_INVALID;
  }
  NR_CHECK_LAUNCH("nr_gemm");
  return NR_OK;
}

template <typename TI, typename TO>
static int launch_gemm256_p16(int epi, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                          const void* W, int64_t ldw, const float* bias, const void* R, int64_t ldr,
                          void* C, int64_t ldc, const EpiArgs& ea, hipStream_t s) {
  dim3 grid((unsigned)(N / G2BN), (unsigned)((M + G2BM - 1) / G2BM));
  const TI* a = (const TI*)A;
  const TI* w = (const TI*)W;
  const TO* r = (const TO*)R;
  TO* c = (TO*)C;
  switch (epi) {
    case NR_EPI_NONE: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_NONE, TO, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RELU: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_RELU, TO, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_EXP: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_EXP, TO, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_GEGLU: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_GEGLU, TO, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RESADD: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_RESADD, TO, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_GELU: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_GELU, TO, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RELU_DROPOUT: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_RELU_DROPOUT, TO, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_DRELU: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_DRELU, TO, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_SOFTMAX64: hipLaunchKernelGGL((gemm256p_kernel<TI, NR_EPI_SOFTMAX64, TO, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    default: set_error("nr_gemm: bad epilogue %d", epi); return NR_ERR_INVALID;
  }
  NR_CHECK_LAUNCH("nr_gemm");
  return NR_OK;
}

// bf16: 16x16x32 MFMA tiles (5-8 % faster than 32x32x16 on the pooler shapes,
// profiles/round1/s2/gemm_mf16_vs_mf32.txt); f32: the exact-f32 32x32x2 tiles.
// Tile order: groups of 4 M-tiles (tile_of; profiles/round1/s5/gemm_group).
constexpr int kGemmGroupM = 4;

template <typename TI, typename TO>
static int launch_gemm256(int epi, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                          const void* W, int64_t ldw, const float* bias, const void* R, int64_t ldr,
                          void* C, int64_t ldc, const EpiArgs& ea, hipStream_t s) {
  EpiArgs eg = ea;
  eg.group_m = kGemmGroupM;
  if (ea.colsum && !(sizeof(TI) == 2 && sizeof(TO) == 2 && persistent_ok(M, N, K, lda, ldw) &&
                     (epi != NR_EPI_DRELU || (((uintptr_t)R & 15) == 0 && ldr % 8 == 0)))) {
    set_error("nr_gemm: column sums need the persistent bf16 kernel (bf16 in/out, K %% 128, 16-byte rows)");
    return NR_ERR_UNSUPPORTED;
  }
  // persistent kernel for bf16 -> bf16 (DRELU reads its forward output in the
  // epilogue's residual window, like RESADD)
  if constexpr (sizeof(TI) == 2 && sizeof(TO) == 2) {
    if (persistent_ok(M, N, K, lda, ldw) && (epi != NR_EPI_DRELU || (((uintptr_t)R & 15) == 0 && ldr % 8 == 0)))
      return launch_gemm256_t(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, eg, s);
    // A past the 32-bit buffer range (e.g. the title encoder's FFN2, [M x 4096]
    // at M > 512 k tokens): persistent launches over row chunks of < 4 GiB of A.
    // A row's K chain and epilogue do not depend on its chunk, so the result is
    // the one-launch result; RELU_DROPOUT's mask hashes the global row index and
    // stays on the tile kernel.
    const int64_t mc = 0xFFFFFFFFll / (2 * lda) / 256 * 256;
    if (epi != NR_EPI_DRELU && epi != NR_EPI_RELU_DROPOUT && mc >= 256 && persistent_ok(mc, N, K, lda, ldw)) {
      for (int64_t m0 = 0; m0 < M; m0 += mc) {
        const int64_t m = M - m0 < mc ? M - m0 : mc;
        const int rc = launch_gemm256_t(epi, m, N, K, static_cast<const char*>(A) + 2 * m0 * lda, lda, W, ldw, bias,
                                        R ? static_cast<const char*>(R) + 2 * m0 * ldr : nullptr, ldr,
                                        static_cast<char*>(C) + 2 * m0 * ldc, ldc, eg, s);
        if (rc != NR_OK) return rc;
      }
      return NR_OK;
    }
  }
  if constexpr (sizeof(TI) == 2) return launch_gemm256_p16<TI, TO>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, eg, s);
  return launch_gemm256_p<TI, TO>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, eg, s);
}

// LayerNorm-folded persistent launch (bf16 in/out; the bf16 latent transform).
int gemm_lnfold_dispatch(int epi, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* W,
                         int64_t ldw, const float* stats, const float* uc, void* C, int64_t ldc, hipStream_t s) {
  NR_CHECK_ARG(epi == NR_EPI_SOFTMAX64 || epi == NR_EPI_GEGLU, "nr_gemm_lnfold: epilogue %d unsupported", epi);
  NR_CHECK_ARG(M >= 0 && N > 0 && K > 0, "nr_gemm_lnfold: bad shape");
  if (M == 0) return NR_OK;
  NR_CHECK_ARG(A && W && C && stats && uc, "nr_gemm_lnfold: null pointer");
  if (N % G2BN != 0 || K % 64 != 0 || !persistent_ok(M, N, K, lda, ldw) || M * 8 > 0xFFFFFFFFll) {
    set_error("nr_gemm_lnfold: unsupported shape M=%lld N=%lld K=%lld", (long long)M, (long long)N, (long long)K);
    return NR_ERR_UNSUPPORTED;
  }
  const int64_t ncols = epi == NR_EPI_GEGLU ? N / 2 : N;
  NR_CHECK_ARG(lda >= K && ldw >= K && lda % 8 == 0 && ldw % 8 == 0 && ldc >= ncols && ldc % 8 == 0 &&
                   ((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)C & 15) == 0 &&
                   ((uintptr_t)stats & 7) == 0 && ((uintptr_t)uc & 3) == 0,
               "nr_gemm_lnfold: operands must be 16-byte aligned with 16-byte row strides");
  const int ntn = (int)(N / G2BN);
  const int64_t ntm = (M + G2BM - 1) / G2BM;
  NR_CHECK_ARG(ntm * ntn <= (1ll << 30), "nr_gemm_lnfold: too many tiles");
  int nt, nh;
  const dim3 grid((unsigned)persistent_schedule(ntm * ntn, &nt, &nh));
  EpiArgs ea{0, 0, 1.f};
  ea.group_m = kGemmGroupM;
  ea.ln_stats = stats;
  ea.ln_uc = uc;
  const __bf16* a = (const __bf16*)A;
  const __bf16* w = (const __bf16*)W;
  __bf16* c = (__bf16*)C;
  if (epi == NR_EPI_GEGLU)
    hipLaunchKernelGGL((gemm256t_kernel<NR_EPI_GEGLU, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, nullptr,
                       nullptr, 0, c, ldc, ea, ntn, (int)ntm, nt, nh);
  else
    hipLaunchKernelGGL((gemm256t_kernel<NR_EPI_SOFTMAX64, true>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw,
                       nullptr, nullptr, 0, c, ldc, ea, ntn, (int)ntm, nt, nh);
  NR_CHECK_LAUNCH("nr_gemm_lnfold");
  return NR_OK;
}

template <typename TI, typename TO>
static int launch_gemm_t(int epi, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                         const void* W, int64_t ldw, const float* bias, const void* R, int64_t ldr,
                         void* C, int64_t ldc, const EpiArgs& ea, hipStream_t s) {
  dim3 grid((unsigned)(N / GBN), (unsigned)((M + GBM - 1) / GBM));
  const TI* a = (const TI*)A;
  const TI* w = (const TI*)W;
  const TO* r = (const TO*)R;
  TO* c = (TO*)C;
  switch (epi) {
    case NR_EPI_NONE: hipLaunchKernelGGL((gemm_kernel<TI, NR_EPI_NONE, TO>), grid, dim3(256), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RELU: hipLaunchKernelGGL((gemm_kernel<TI, NR_EPI_RELU, TO>), grid, dim3(256), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_EXP: hipLaunchKernelGGL((gemm_kernel<TI, NR_EPI_EXP, TO>), grid, dim3(256), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_GEGLU: hipLaunchKernelGGL((gemm_kernel<TI, NR_EPI_GEGLU, TO>), grid, dim3(256), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RESADD: hipLaunchKernelGGL((gemm_kernel<TI, NR_EPI_RESADD, TO>), grid, dim3(256), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_GELU: hipLaunchKernelGGL((gemm_kernel<TI, NR_EPI_GELU, TO>), grid, dim3(256), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RELU_DROPOUT: hipLaunchKernelGGL((gemm_kernel<TI, NR_EPI_RELU_DROPOUT, TO>), grid, dim3(256), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_DRELU: hipLaunchKernelGGL((gemm_kernel<TI, NR_EPI_DRELU, TO>), grid, dim3(256), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    default: set_error("nr_gemm: bad epilogue %d", epi); return NR_ERR_INVALID;
  }
  NR_CHECK_LAUNCH("nr_gemm");
  return NR_OK;
}

int gemm_dispatch(int dtype_in, int dtype_out, int epi, int64_t M, int64_t N, int64_t K,
                  const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
                  const void* R, int64_t ldr, void* C, int64_t ldc, hipStream_t s) {
  return gemm_dispatch_ex(dtype_in, dtype_out, epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc,
                          EpiArgs{0, 0, 1.f}, s);
}

int gemm_dispatch_ex(int dtype_in, int dtype_out, int epi, int64_t M, int64_t N, int64_t K,
                     const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
                     const void* R, int64_t ldr, void* C, int64_t ldc, const EpiArgs& ea, hipStream_t s) {
  NR_CHECK_ARG(dtype_in == NR_F32 || dtype_in == NR_BF16, "nr_gemm: bad dtype_in %d", dtype_in);
  NR_CHECK_ARG(dtype_out == NR_F32 || dtype_out == NR_BF16, "nr_gemm: bad dtype_out %d", dtype_out);
  NR_CHECK_ARG(M >= 0 && N > 0 && K > 0, "nr_gemm: bad shape M=%lld N=%lld K=%lld", (long long)M, (long long)N, (long long)K);
  if (M == 0) return NR_OK;
  const int64_t bk = dtype_in == NR_F32 ? 32 : 64;
  if (N % GBN != 0 || K % bk != 0) {
    set_error("nr_gemm: unsupported shape N=%lld (need %%128) K=%lld (need %%%lld)", (long long)N, (long long)K, (long long)bk);
    return NR_ERR_UNSUPPORTED;
  }
  NR_CHECK_ARG(A && W && C, "nr_gemm: null operand");
  NR_CHECK_ARG((epi != NR_EPI_RESADD && epi != NR_EPI_DRELU && epi != NR_EPI_SOFTMAX64_BWD) || R,
               "nr_gemm: RESADD/DRELU/SOFTMAX64_BWD need R");
  NR_CHECK_ARG(epi >= NR_EPI_NONE && epi <= NR_EPI_SOFTMAX64_BWD, "nr_gemm: bad epilogue %d", epi);
  if (epi == NR_EPI_SOFTMAX64_BWD &&
      !(dtype_in == NR_BF16 && dtype_out == NR_BF16 && N % G2BN == 0 && persistent_ok(M, N, K, lda, ldw) &&
        ((uintptr_t)C & 15) == 0 && ldc % 8 == 0 && ((uintptr_t)R & 15) == 0 && ldr % 8 == 0)) {
    set_error("nr_gemm: SOFTMAX64_BWD runs on the persistent bf16 kernel only (bf16 in/out, N %% 256, K >= 128, "
              "16-byte aligned rows)");
    return NR_ERR_UNSUPPORTED;
  }
  const int64_t e16 = dtype_in == NR_F32 ? 4 : 8;  // elements per 16 B
  NR_CHECK_ARG(lda >= K && ldw >= K && lda % e16 == 0 && ldw % e16 == 0 &&
                   ((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0,
               "nr_gemm: A/W must be 16-byte aligned with 16-byte row strides");
  const int64_t ncols = epi == NR_EPI_GEGLU ? N / 2 : N;
  NR_CHECK_ARG(ldc >= ncols, "nr_gemm: ldc too small");
  NR_CHECK_ARG((M + GBM - 1) / GBM <= 65535, "nr_gemm: M too large (> 8.3M rows)");
  // 256x256 glds kernel when the shape allows (every pooler GEMM); the
  // 128x128 register-staged kernel covers N % 256 != 0 and unaligned outputs.
  const int64_t vo = dtype_out == NR_F32 ? 4 : 8;  // the LDS-staged epilogue stores 16 B per lane
  const bool aligned_out = ((uintptr_t)C & 15) == 0 && ldc % vo == 0 &&
                           ((epi != NR_EPI_RESADD && epi != NR_EPI_DRELU) || (((uintptr_t)R & 15) == 0 && ldr % vo == 0));
  const bool big = (N % G2BN == 0) && aligned_out;
  if (epi == NR_EPI_SOFTMAX64 && !big) {
    set_error("nr_gemm: SOFTMAX64 needs N %% 256 == 0 and 16-byte aligned output rows");
    return NR_ERR_UNSUPPORTED;
  }
  if (dtype_in == NR_F32) {
    if (big) {
      if (dtype_out == NR_F32) return launch_gemm256<float, float>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, ea, s);
      return launch_gemm256<float, __bf16>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, ea, s);
    }
    if (dtype_out == NR_F32) return launch_gemm_t<float, float>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, ea, s);
    return launch_gemm_t<float, __bf16>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, ea, s);
  }
  if (big) {
    if (dtype_out == NR_F32) return launch_gemm256<__bf16, float>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, ea, s);
    return launch_gemm256<__bf16, __bf16>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, ea, s);
  }
  if (dtype_out == NR_F32) return launch_gemm_t<__bf16, float>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, ea, s);
  return launch_gemm_t<__bf16, __bf16>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, ea, s);
}

}  // namespace nr

extern "C" int nr_gemm_relu_dropout(int dtype_in, int dtype_out, int64_t M, int64_t N, int64_t K,
                                    const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
                                    void* C, int64_t ldc, uint64_t seed, float p, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(p >= 0.f && p < 1.f, "nr_gemm_relu_dropout: p must be in [0, 1)");
  if (M > 0) NR_CHECK_DEVICE("nr_gemm_relu_dropout", A, W, bias, C);
  const uint32_t thr = nr::dropout_threshold(p);
  return nr::gemm_dispatch_ex(dtype_in, dtype_out, NR_EPI_RELU_DROPOUT, M, N, K, A, lda, W, ldw, bias, nullptr, 0,
                              C, ldc, nr::EpiArgs{seed, thr, 1.0f / (1.0f - p)}, (hipStream_t)stream);
}

extern "C" int nr_gemm_drelu(int dtype_in, int dtype_out, int64_t M, int64_t N, int64_t K, const void* A,
                             int64_t lda, const void* W, int64_t ldw, const void* Y, int64_t ldy, void* C,
                             int64_t ldc, float scale, void* stream) {
  nr::clear_error();
  if (M > 0) NR_CHECK_DEVICE("nr_gemm_drelu", A, W, Y, C);
  return nr::gemm_dispatch_ex(dtype_in, dtype_out, NR_EPI_DRELU, M, N, K, A, lda, W, ldw, nullptr, Y, ldy, C, ldc,
                              nr::EpiArgs{0, 0, scale}, (hipStream_t)stream);
}

extern "C" int nr_gemm(int dtype_in, int dtype_out, int epilogue, int64_t M, int64_t N, int64_t K,
                       const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
                       const void* R, int64_t ldr, void* C, int64_t ldc, void* stream) {
  nr::clear_error();
  if (M > 0) NR_CHECK_DEVICE("nr_gemm", A, W, bias, R, C);
  return nr::gemm_dispatch(dtype_in, dtype_out, epilogue, M, N, K, A, lda, W, ldw, bias, R, ldr, C,
                           ldc, (hipStream_t)stream);
}

extern "C" int nr_gemm_grouped_tn(int dtype_out, int n, const int64_t* M, const int64_t* N, const int64_t* K,
                                  const void* const* A, const int64_t* lda, const void* const* W, const int64_t* ldw,
                                  void* const* C, const int64_t* ldc, const float* alpha, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(n >= 1 && n <= NR_GEMM_MAX_GROUP, "nr_gemm_grouped_tn: n=%d outside [1, %d]", n, NR_GEMM_MAX_GROUP);
  NR_CHECK_ARG(M && N && K && A && lda && W && ldw && C && ldc, "nr_gemm_grouped_tn: null array");
  nr::GemmProblem p[NR_GEMM_MAX_GROUP];
  for (int i = 0; i < n; ++i) {
    if (K[i] > 0) NR_CHECK_DEVICE("nr_gemm_grouped_tn", A[i], W[i], C[i]);
    p[i] = nr::GemmProblem{M[i], N[i], K[i], A[i], lda[i], 0, W[i], ldw[i], 0, C[i], ldc[i], 0, 1,
                           alpha ? alpha[i] : 1.0f};
  }
  return nr::gemm_group_tn_dispatch(dtype_out, p, n, (hipStream_t)stream);
}

extern "C" int nr_gemm_grouped(int dtype_in, int dtype_out, int n, const int64_t* M, const int64_t* N,
                               const int64_t* K, const void* const* A, const int64_t* lda, const void* const* W,
                               const int64_t* ldw, void* const* C, const int64_t* ldc, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(n >= 1 && n <= NR_GEMM_MAX_GROUP, "nr_gemm_grouped: n=%d outside [1, %d]", n, NR_GEMM_MAX_GROUP);
  NR_CHECK_ARG(M && N && K && A && lda && W && ldw && C && ldc, "nr_gemm_grouped: null array");
  nr::GemmProblem p[NR_GEMM_MAX_GROUP];
  for (int i = 0; i < n; ++i) {
    if (M[i] > 0) NR_CHECK_DEVICE("nr_gemm_grouped", A[i], W[i], C[i]);
    p[i] = nr::GemmProblem{M[i], N[i], K[i], A[i], lda[i], 0, W[i], ldw[i], 0, C[i], ldc[i], 0, 1, 1.0f};
  }
  return nr::gemm_group_dispatch(dtype_in, dtype_out, p, n, (hipStream_t)stream);
}
