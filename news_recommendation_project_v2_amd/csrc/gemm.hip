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

#include <stdlib.h>

#ifndef NR_GEMM_EPI_BLOCK_SYNC
#define NR_GEMM_EPI_BLOCK_SYNC 0  // A/B build switch: workgroup barriers between epilogue passes
#endif
#ifndef NR_GEMM_STAMPS
#define NR_GEMM_STAMPS 0  // diagnostic build switch: per-block phase stamps (tools/gemm_stamps.py)
#endif
#ifndef NR_GEMM_SLAB16
#define NR_GEMM_SLAB16 0  // A/B build switch: bf16 epilogue slab for pointwise epilogues (measured slower)
#endif
#ifndef NR_GEMM_NT_STORE
#define NR_GEMM_NT_STORE 0  // A/B build switch: non-temporal epilogue stores
#endif

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

// Extra epilogue arguments (dropout of the training forward; unused otherwise).
struct EpiArgs {
  uint64_t seed;  // dropout stream
  uint32_t thr;   // drop iff drop_hash(seed, row * N + col) < thr  (thr = p * 2^32)
  float scale;    // 1 / (1 - p)
  int group_m = 1;  // 256x256 tile order: >1 groups group_m M-tiles (see tile_of)
};

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
              v = drop_hash(ea.seed, (uint64_t)(row * N + col)) < ea.thr ? 0.f : fmaxf(v, 0.f) * ea.scale;
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
  // The slabs overlay the operand stages: one workgroup barrier so that no
  // wave still reads operands; after it each wave only touches its own slab,
  // so the passes order their LDS traffic wave-locally (no further workgroup
  // barriers: waves drift apart and their store bursts spread out).
#if NR_GEMM_EPI_BLOCK_SYNC
#define NR_EPI_SYNC() __syncthreads()
#else
  __syncthreads();
#define NR_EPI_SYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#endif
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
  // bf16 output of a pointwise epilogue on 16x16 tiles: the slab holds the
  // final bf16 values (half the LDS round trip).  A lane's 4 rows of one
  // column are paired with the neighbour lane's column by one DPP swap so each
  // LDS write is a 2-column bf16 dword; dwords XOR-swizzled by row pair so the
  // 32 lanes of a write hit distinct banks (COLS 64; 2-way for GEGLU's 32).
  constexpr bool SLAB16 = MF16 && NR_GEMM_SLAB16 && sizeof(TO) == 2 &&
                          (EPI == NR_EPI_NONE || EPI == NR_EPI_RELU || EPI == NR_EPI_EXP || EPI == NR_EPI_GELU ||
                           EPI == NR_EPI_GEGLU || EPI == NR_EPI_RELU_DROPOUT);
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if constexpr (SLAB16) {
      constexpr int DW = COLS / 2;  // dwords per slab row
      uint32_t* s32 = reinterpret_cast<uint32_t*>(slab);
      auto sidx = [](int row, int dw) {
        const int x = DW == 32 ? ((row >> 1) & 3) << 3 : ((row >> 1) & 1) << 3;
        return row * DW + (dw ^ x);
      };
      const int c16 = lane & 15, r16 = 4 * (lane >> 4);
      const bool odd = lane & 1;
      constexpr int NOUT = (EPI == NR_EPI_GEGLU) ? 2 : 4;  // 16-column output groups per wave
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mi = 4 * pass + i;
#pragma unroll
        for (int ni = 0; ni < NOUT; ++ni) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if constexpr (EPI == NR_EPI_GEGLU) {
              v[r] = (acc[mi][ni][r] + b16[ni]) * gelu_erf(acc[mi][ni + 2][r] + b16[ni + 2]);
            } else {
              float x = acc[mi][ni][r] + b16[ni];
              if constexpr (EPI == NR_EPI_RELU) x = fmaxf(x, 0.f);
              if constexpr (EPI == NR_EPI_RELU_DROPOUT) {
                const uint64_t gi = (uint64_t)((m0 + wm * 128 + pass * 64 + 16 * i + r16 + r) * N + wcol + 16 * ni + c16);
                x = drop_hash(ea.seed, gi) < ea.thr ? 0.f : fmaxf(x, 0.f) * ea.scale;
              }
              if constexpr (EPI == NR_EPI_EXP) x = expf(x);
              if constexpr (EPI == NR_EPI_GELU) x = gelu_erf(x);
              v[r] = x;
            }
          }
          // even lane keeps rows 0-1 and receives the odd neighbour's rows 0-1; odd keeps rows 2-3
          const float x0 = odd ? v[0] : v[2], x1 = odd ? v[1] : v[3];
          const float y0 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x0), 0xB1, 0xF, 0xF, false));
          const float y1 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x1), 0xB1, 0xF, 0xF, false));
          const float lo0 = odd ? y0 : v[0], hi0 = odd ? v[2] : y0;
          const float lo1 = odd ? y1 : v[1], hi1 = odd ? v[3] : y1;
          const int row0 = 16 * i + r16 + (odd ? 2 : 0);
          const int dw = (16 * ni + (c16 & ~1)) >> 1;
          const uint32_t p0 = (uint32_t)__builtin_bit_cast(unsigned short, (__bf16)lo0) |
                              ((uint32_t)__builtin_bit_cast(unsigned short, (__bf16)hi0) << 16);
          const uint32_t p1 = (uint32_t)__builtin_bit_cast(unsigned short, (__bf16)lo1) |
                              ((uint32_t)__builtin_bit_cast(unsigned short, (__bf16)hi1) << 16);
          s32[sidx(row0, dw)] = p0;
          s32[sidx(row0 + 1, dw)] = p1;
        }
      }
      NR_EPI_SYNC();
      constexpr int LPR16 = DW / 4;     // lanes per row (16 B each)
      constexpr int RPI16 = 64 / LPR16;  // rows per wave instruction
      const int rr16 = lane / LPR16, cd = (lane % LPR16) * 4;
#pragma unroll
      for (int it = 0; it < 64 / RPI16; ++it) {
        const int lr = it * RPI16 + rr16;
        const int64_t row = m0 + wm * 128 + pass * 64 + lr;
        const uint4 q = *reinterpret_cast<const uint4*>(s32 + sidx(lr, cd));
        if (row < M) *reinterpret_cast<uint4*>(C + row * ldc + ocol0 + 2 * cd) = q;
      }
      NR_EPI_SYNC();
      continue;
    }
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
              if constexpr (EPI == NR_EPI_RELU) v = fmaxf(v, 0.f);
              if constexpr (EPI == NR_EPI_RELU_DROPOUT) {
                const uint64_t gi = (uint64_t)((m0 + wm * 128 + pass * 64 + lr) * N + wcol + 16 * ni + c16);
                v = drop_hash(ea.seed, gi) < ea.thr ? 0.f : fmaxf(v, 0.f) * ea.scale;
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
          if constexpr (EPI == NR_EPI_RELU) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); }
          if constexpr (EPI == NR_EPI_RELU_DROPOUT) {
            const uint64_t gi = (uint64_t)((m0 + wm * 128 + pass * 64 + lr) * N + wcol + cl);
            v0 = drop_hash(ea.seed, gi) < ea.thr ? 0.f : fmaxf(v0, 0.f) * ea.scale;
            v1 = drop_hash(ea.seed, gi + 32) < ea.thr ? 0.f : fmaxf(v1, 0.f) * ea.scale;
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
#if NR_GEMM_NT_STORE
        __builtin_nontemporal_store(*reinterpret_cast<const f32x4*>(o), reinterpret_cast<f32x4*>(C + row * ldc + ocol0 + cc));
#else
        *reinterpret_cast<uint4*>(C + row * ldc + ocol0 + cc) = *reinterpret_cast<const uint4*>(o);
#endif
      }
    }
    NR_EPI_SYNC();
  }
#undef NR_EPI_SYNC
}

template <typename TI, int EPI, typename TO>
__global__ __launch_bounds__(512, 2) void gemm256_kernel(int64_t M, int64_t N, int64_t K,
                                                             const TI* __restrict__ A, int64_t lda,
                                                             const TI* __restrict__ W, int64_t ldw,
                                                             const float* __restrict__ bias, const TO* R,
                                                             int64_t ldr, TO* C, int64_t ldc, EpiArgs ea) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * G2_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int64_t n0 = (int64_t)blockIdx.x * G2BN;
  const int64_t m0 = (int64_t)blockIdx.y * G2BM;

  // glds source pointers: wave issues 4 A + 4 B instructions per K tile, each
  // filling 8 rows x 128 B; lane l fills (row R0 + l/8, LDS chunk l%8).
  constexpr int BK = 128 / (int)sizeof(TI), CE = 16 / (int)sizeof(TI);
  const TI* asrc[4];
  const TI* bsrc[4];
  int ldsoff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r0 = (wave * 4 + j) * 8;
    const int row = r0 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    const int64_t ar = min(m0 + row, M - 1);
    asrc[j] = A + ar * lda + chunk * CE;
    bsrc[j] = W + (n0 + row) * ldw + chunk * CE;
    ldsoff[j] = r0 * 128;
  }
  auto issue = [&](int stage, int64_t kt) {
    unsigned char* sa = smem + stage * G2_STAGE;
    unsigned char* sb = sa + G2BM * 128;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      __builtin_amdgcn_global_load_lds((g_void*)(asrc[j] + kt * BK), (lds_void*)(sa + ldsoff[j]), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((g_void*)(bsrc[j] + kt * BK), (lds_void*)(sb + ldsoff[j]), 16, 0, 0);
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
  int aoff[4], boff[2], asw[4], bsw[2];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int row = wm * 128 + mi * 32 + fr;
    aoff[mi] = row * 128;
    asw[mi] = (row >> 1) & 7;
  }
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const int row = wn * 64 + ni * 32 + fr;
    boff[ni] = G2BM * 128 + row * 128;
    bsw[ni] = (row >> 1) & 7;
  }

  auto compute = [&](int stage) {
    const unsigned char* s = smem + stage * G2_STAGE;
    if constexpr (sizeof(TI) == 2) {
      // 32x32x16 bf16: lane (r, h) holds k = 16ks + 8h + j (chunk 2ks + h) of row r
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int c = 2 * ks + fh;
        bf16x8 af[4], bfr[2];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) af[mi] = *reinterpret_cast<const bf16x8*>(s + aoff[mi] + ((c ^ asw[mi]) << 4));
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) bfr[ni] = *reinterpret_cast<const bf16x8*>(s + boff[ni] + ((c ^ bsw[ni]) << 4));
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
      }
    } else {
      // 32x32x2 f32: lane half h covers k = 16h + 4q + t (chunk 4h + q), A and W alike
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 4 * fh + q;
        f32x4 af[4], bfr[2];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) af[mi] = *reinterpret_cast<const f32x4*>(s + aoff[mi] + ((c ^ asw[mi]) << 4));
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) bfr[ni] = *reinterpret_cast<const f32x4*>(s + boff[ni] + ((c ^ bsw[ni]) << 4));
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi][t], bfr[ni][t], acc[mi][ni], 0, 0, 0);
      }
    }
  };

  const int64_t nk = K / BK;
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) issue((int)((kt + 1) & 1), kt + 1);
    compute((int)(kt & 1));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  gemm256_store<EPI, TO>(acc, smem, wave, lane, wm, wn, m0, n0, M, N, bias, R, ldr, C, ldc, ea);
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
// Same LDS images, swizzle and epilogue as gemm256_kernel.
// XCD-aware bijective remap of the launch order: dispatch slot `orig` runs on
// XCD orig % 8; consecutive output tiles (the N tiles sharing an A panel) are
// given to one XCD so its L2 holds the panel.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
  return (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
}

#if NR_GEMM_STAMPS
// Diagnostic build only (-DNR_GEMM_STAMPS=1, tools/gemm_stamps.py): per-block
// s_memrealtime stamps of the 256x256 kernel's phases, written by lanes 0-7 of
// wave 0 into a buffer nothing else reads.
__device__ unsigned long long* g_gemm_stamps = nullptr;
#endif

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

template <typename TI, int EPI, typename TO, bool MF16>
__device__ __forceinline__ void gemm256p_body(unsigned char* smem, int64_t m0, int64_t n0, int64_t M, int64_t N,
                                              int64_t K, const TI* __restrict__ A, int64_t lda,
                                              const TI* __restrict__ W, int64_t ldw, const float* __restrict__ bias,
                                              const TO* R, int64_t ldr, TO* C, int64_t ldc, const EpiArgs& ea) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;

  constexpr int BK = 128 / (int)sizeof(TI), CE = 16 / (int)sizeof(TI);
  // half-tile DMA sources: wave covers rows 128h + 16 wave + 8 j + lane / 8
  const TI* asrc[2][2];
  const TI* bsrc[2][2];
  int hoff[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r0 = 128 * h + (wave * 2 + j) * 8;
      const int row = r0 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      asrc[h][j] = A + min(m0 + row, M - 1) * lda + chunk * CE;
      bsrc[h][j] = W + (n0 + row) * ldw + chunk * CE;
      hoff[h][j] = r0 * 128;
    }
  auto dmaA = [&](int h, int stage, int64_t kt) {
    unsigned char* sa = smem + stage * G2_STAGE;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((g_void*)(asrc[h][j] + kt * BK), (lds_void*)(sa + hoff[h][j]), 16, 0, 0);
  };
  auto dmaB = [&](int h, int stage, int64_t kt) {
    unsigned char* sb = smem + stage * G2_STAGE + G2BM * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((g_void*)(bsrc[h][j] + kt * BK), (lds_void*)(sb + hoff[h][j]), 16, 0, 0);
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
  auto readA = [&](int stage, int qm) {
    const unsigned char* s = smem + stage * G2_STAGE;
#pragma unroll
    for (int i = 0; i < QA; ++i)
#pragma unroll
      for (int f = 0; f < NF; ++f)
        fa[i][f] = *reinterpret_cast<const frag_t*>(s + aoff[QA * qm + i] + ((chunk_of(f) ^ asw[QA * qm + i]) << 4));
  };
  auto readB = [&](int stage, int qn, frag_t (&fb)[QB][NF]) {
    const unsigned char* s = smem + stage * G2_STAGE;
#pragma unroll
    for (int j = 0; j < QB; ++j)
#pragma unroll
      for (int f = 0; f < NF; ++f)
        fb[j][f] = *reinterpret_cast<const frag_t*>(s + boff[QB * qn + j] + ((chunk_of(f) ^ bsw[QB * qn + j]) << 4));
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
#if NR_GEMM_STAMPS
  const unsigned long long st0 = __builtin_amdgcn_s_memrealtime();
#endif
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
#if NR_GEMM_STAMPS
  const unsigned long long st1 = __builtin_amdgcn_s_memrealtime();
#endif
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
#if NR_GEMM_STAMPS
  const unsigned long long st2 = __builtin_amdgcn_s_memrealtime();
#endif
  gemm256_store<EPI, TO, MF16>(acc, smem, wave, lane, wm, wn, m0, n0, M, N, bias, R, ldr, C, ldc, ea);
#if NR_GEMM_STAMPS
  const unsigned long long st3 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long st4 = __builtin_amdgcn_s_memrealtime();
  if (wave == 0 && lane < 8 && g_gemm_stamps) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20); // XCC_ID
    const unsigned long long v[8] = {st0, st1, st2, st3, st4, hw, xcc, (unsigned long long)(m0 << 20 | n0)};
    unsigned long long x = v[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) x = lane == i ? v[i] : x;
    g_gemm_stamps[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + lane] = x;
  }
#endif
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

// Grouped launch of up to NR_GEMM_MAX_GROUP independent problems with one
// dtype / epilogue (no bias, no residual): one grid over all problems' tiles,
// so small problems (the config-5 weight-grad GEMMs, 64 tiles each) fill the
// 256 CUs together instead of one after another.  tile_end[p] = prefix sum of
// the problems' tile counts; tiles are remapped XCD-aware over the whole grid,
// so one problem's N tiles of an A panel stay on one XCD.
struct GemmGroup {
  int n;
  int tile_end[NR_GEMM_MAX_GROUP];
  int ntn[NR_GEMM_MAX_GROUP];
  int64_t M[NR_GEMM_MAX_GROUP], N[NR_GEMM_MAX_GROUP], K[NR_GEMM_MAX_GROUP];
  const void* A[NR_GEMM_MAX_GROUP];
  const void* W[NR_GEMM_MAX_GROUP];
  void* C[NR_GEMM_MAX_GROUP];
  int64_t lda[NR_GEMM_MAX_GROUP], ldw[NR_GEMM_MAX_GROUP], ldc[NR_GEMM_MAX_GROUP];
};

template <typename TI, typename TO, bool MF16>
__global__ __launch_bounds__(512, 2) void gemm256p_group_kernel(GemmGroup g) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * G2_STAGE];
  const int t = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  int p = 0;
  while (p + 1 < g.n && t >= g.tile_end[p]) ++p;
  const int local = t - (p ? g.tile_end[p - 1] : 0);
  const int nx = g.ntn[p];
  gemm256p_body<TI, NR_EPI_NONE, TO, MF16>(smem, (int64_t)(local / nx) * G2BM, (int64_t)(local % nx) * G2BN, g.M[p],
                                           g.N[p], g.K[p], (const TI*)g.A[p], g.lda[p], (const TI*)g.W[p], g.ldw[p],
                                           nullptr, nullptr, 0, (TO*)g.C[p], g.ldc[p], EpiArgs{0, 0, 1.f});
}

// ---------------------------------------------------------------------------
// Persistent bf16 variant (16x16x32 MFMA tiles): one 512-thread workgroup per
// CU walks its share of the 256x256 output tiles.  The main loop is
// gemm256p_kernel's; what changes is the tile boundary: as soon as a tile's K
// loop ends, the NEXT tile's prologue DMAs (K tile 0, and K tile 1's B halves)
// are issued into the two operand stages, and the finished tile's epilogue
// runs from a separate 32 KiB LDS region (a 4 KiB, 16-row slab per wave) while
// they fly.  With one workgroup per CU (234 VGPRs, 160 KiB LDS) the prologue
// latency and the epilogue (GEGLU's erf, stores) would otherwise be exposed
// once per tile: at K = 512-1024 that is 10-20 % of a tile.  Tiles are split
// into 8 contiguous ranges, one per XCD (workgroups b = x mod 8), so the tiles
// an XCD runs concurrently share A panels in its L2.
template <int EPI, typename TO>
__device__ __forceinline__ void epi16_store(const f32x4 (&acc)[8][4], float* slab, int lane, int wm, int wn,
                                            int64_t m0, int64_t n0, int64_t M, int64_t N,
                                            const float (&b16)[4], const TO* R, int64_t ldr, TO* C,
                                            int64_t ldc, const EpiArgs& ea) {
  constexpr int COLS = (EPI == NR_EPI_GEGLU) ? 32 : 64;
  constexpr int VEC = 16 / (int)sizeof(TO);
  constexpr int LPR = COLS / VEC;
  constexpr int RPI = 64 / LPR;
  constexpr int ITS = 16 / RPI;
  const int64_t wcol = n0 + wn * 64;
  const int64_t ocol0 = (EPI == NR_EPI_GEGLU) ? wcol / 2 : wcol;
  const int c16 = lane & 15, r16 = 4 * (lane >> 4);
  // slab [16][COLS] f32; column bit 4 flipped on rows 4-7 / 12-15 so the two
  // 16-lane halves of a 32-lane store group hit different banks
  auto sidx = [](int row, int col) { return row * COLS + (col ^ ((row & 4) << 2)); };
  const int rr = lane / LPR, cc = (lane % LPR) * VEC;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r16 + r;
      if constexpr (EPI == NR_EPI_GEGLU) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          slab[sidx(row, 16 * ni + c16)] = (acc[mi][ni][r] + b16[ni]) * gelu_erf(acc[mi][ni + 2][r] + b16[ni + 2]);
      } else {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          float v = acc[mi][ni][r] + b16[ni];
          if constexpr (EPI == NR_EPI_RELU) v = fmaxf(v, 0.f);
          if constexpr (EPI == NR_EPI_RELU_DROPOUT) {
            const uint64_t gi = (uint64_t)((m0 + wm * 128 + mi * 16 + row) * N + wcol + 16 * ni + c16);
            v = drop_hash(ea.seed, gi) < ea.thr ? 0.f : fmaxf(v, 0.f) * ea.scale;
          }
          if constexpr (EPI == NR_EPI_EXP) v = expf(v);
          if constexpr (EPI == NR_EPI_GELU) v = gelu_erf(v);
          slab[sidx(row, 16 * ni + c16)] = v;
        }
      }
    }
#pragma unroll
    for (int it = 0; it < ITS; ++it) {
      const int lr = it * RPI + rr;
      const int64_t row = m0 + wm * 128 + mi * 16 + lr;
      float v[VEC];
#pragma unroll
      for (int q = 0; q < VEC; q += 4) {
        const float4 f = *reinterpret_cast<const float4*>(slab + sidx(lr, cc + q));
        v[q] = f.x; v[q + 1] = f.y; v[q + 2] = f.z; v[q + 3] = f.w;
      }
      if constexpr (EPI == NR_EPI_SOFTMAX64) {
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
          float rf[VEC];
          if constexpr (sizeof(TO) == 4) {
            rf[0] = __uint_as_float(rv.x); rf[1] = __uint_as_float(rv.y);
            rf[2] = __uint_as_float(rv.z); rf[3] = __uint_as_float(rv.w);
          } else {
            const uint32_t w4[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) { rf[2 * q] = bf16_lo(w4[q]); rf[2 * q + 1] = bf16_hi(w4[q]); }
          }
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            if constexpr (EPI == NR_EPI_RESADD) v[q] += rf[q];
            else v[q] = rf[q] > 0.f ? v[q] * ea.scale : 0.f;
          }
        }
        TO o[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) o[q] = to_out<TO>(v[q]);
        *reinterpret_cast<uint4*>(C + row * ldc + ocol0 + cc) = *reinterpret_cast<const uint4*>(o);
      }
    }
  }
}

constexpr int G2_EPI_SLAB = 16 * 64 * 4;  // bytes per wave

template <int EPI, typename TO>
__global__ __launch_bounds__(512, 2) void gemm256pp_kernel(int64_t M, int64_t N, int64_t K,
                                                           const __bf16* __restrict__ A, int64_t lda,
                                                           const __bf16* __restrict__ W, int64_t ldw,
                                                           const float* __restrict__ bias, const TO* R,
                                                           int64_t ldr, TO* C, int64_t ldc, EpiArgs ea,
                                                           int tiles_n, int n_tiles) {
  typedef __bf16 TI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * G2_STAGE + 8 * G2_EPI_SLAB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int wmu = __builtin_amdgcn_readfirstlane(wm);
  float* slab = reinterpret_cast<float*>(smem + 2 * G2_STAGE + wave * G2_EPI_SLAB);

  // tile schedule: XCD group x = blockIdx % 8 owns a contiguous range of tiles
  const int G = (int)gridDim.x;
  int t, t_end, t_step;
  if (G % 8 == 0 && G >= 8) {
    const int x = (int)blockIdx.x & 7, li = (int)blockIdx.x >> 3;
    const int q = n_tiles >> 3, r = n_tiles & 7;
    const int lo = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    t = lo + li;
    t_end = lo + q + (x < r ? 1 : 0);
    t_step = G >> 3;
  } else {
    t = (int)blockIdx.x;
    t_end = n_tiles;
    t_step = G;
  }
  if (t >= t_end) return;  // workgroup-uniform

  constexpr int BK = 64, CE = 8;
  // DMA addressing recomputed per issue from tile-uniform m0/n0 and a few
  // lane constants (keeps ~16 VGPRs of 64-bit pointers out of the persistent
  // loop).  Lane l of wave w fills row 128h + 16w + 8j + l/8, 16-B chunk
  // (l & 7) ^ ((4j + l/16) & 7) of the swizzled image (= chunk ^ (row>>1 & 7)).
  int64_t tm0 = 0, tn0 = 0;
  const int rl = 16 * wave + (lane >> 3);
  auto cj = [&](int j) { return (lane & 7) ^ ((4 * j + (lane >> 4)) & 7); };
  auto dmaA = [&](int h, int stage, int64_t kt) {
    unsigned char* sa = smem + stage * G2_STAGE;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t row = min(tm0 + 128 * h + 8 * j + rl, M - 1);
      const TI* src = A + row * lda + cj(j) * CE + kt * BK;
      __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(sa + (128 * h + 16 * wave + 8 * j) * 128), 16, 0, 0);
    }
  };
  auto dmaB = [&](int h, int stage, int64_t kt) {
    unsigned char* sb = smem + stage * G2_STAGE + G2BM * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const TI* src = W + (tn0 + 128 * h + 8 * j + rl) * ldw + cj(j) * CE + kt * BK;
      __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(sb + (128 * h + 16 * wave + 8 * j) * 128), 16, 0, 0);
    }
  };
  auto setup = [&](int tile) {
    tn0 = (int64_t)(tile % tiles_n) * G2BN;
    tm0 = (int64_t)(tile / tiles_n) * G2BM;
  };
  const int64_t nk = K / BK;
  auto prologue = [&]() {
    dmaB(0, 0, 0);
    dmaB(1, 0, 0);
    dmaA(0, 0, 0);
    dmaA(1, 0, 0);
    if (nk > 1) {
      dmaB(0, 1, 1);
      dmaB(1, 1, 1);
    }
  };

  // fragment addresses: 16x16x32 tiles; the swizzle term (row >> 1) & 7 is
  // the same for every tile of a lane (tiles are 16 rows apart)
  const int c16 = lane & 15;
  const int sw = (c16 >> 1) & 7;
  const int abase = (wm * 128 + c16) * 128;
  const int bbase = G2BM * 128 + (wn * 64 + c16) * 128;
  const int cf0 = ((0 + (lane >> 4)) ^ sw) << 4, cf1 = ((4 + (lane >> 4)) ^ sw) << 4;
  typedef f32x4 frag_t;
  frag_t fa[4][2], fb0[2][2], fb1[2][2];
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
  auto mma = [&](int qm, int qn, const frag_t (&fb)[2][2]) {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 * qm + i][2 * qn + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, fa[i][f]), __builtin_bit_cast(bf16x8, fb[j][f]), acc[4 * qm + i][2 * qn + j],
              0, 0, 0);
  };
#define NR_PHASE_SYNC_MMA(QM, NI, FB)                   \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
  __builtin_amdgcn_sched_barrier(0);                   \
  __builtin_amdgcn_s_barrier();                        \
  __builtin_amdgcn_s_setprio(1);                       \
  mma(QM, NI, FB);                                     \
  __builtin_amdgcn_s_setprio(0);                       \
  __builtin_amdgcn_s_barrier();

  // The epilogue of a full tile issues exactly EPI_STORES 16-byte stores per
  // wave AFTER the next tile's prologue DMAs; vmcnt retires loads, stores and
  // LDS-DMA in issue order (MI355X_MICROARCH: one counter, issue order), so
  // vmcnt(EPI_STORES) means "the prologue has landed" while the previous
  // tile's stores drain under this tile's MFMAs.  After a ragged (M-tail)
  // tile fewer stores were issued: drain everything.
  constexpr int EPI_COLS = (EPI == NR_EPI_GEGLU) ? 32 : 64;
  constexpr int EPI_STORES = 8 * (16 / (64 / (EPI_COLS / (16 / (int)sizeof(TO)))));
  static_assert(EPI_STORES == 8 || EPI_STORES == 16 || EPI_STORES == 32, "epilogue store count");
  setup(t);
  prologue();
  bool drain_all = true;
  while (true) {
    if (drain_all) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (EPI_STORES == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (EPI_STORES == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wmu == 1) __builtin_amdgcn_s_barrier();  // stagger the wave groups
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[mi][ni][r] = 0.f;
    for (int64_t kt = 0; kt < nk; ++kt) {
      const int st = (int)(kt & 1), ns = st ^ 1;
      const bool pre1 = kt + 1 < nk, pre2 = kt + 2 < nk;
      readA(st, 0);
      readB(st, 0, fb0);
      if (pre1) dmaA(0, ns, kt + 1);
      NR_PHASE_SYNC_MMA(0, 0, fb0)
      readB(st, 1, fb1);
      if (pre1) dmaA(1, ns, kt + 1);
      NR_PHASE_SYNC_MMA(0, 1, fb1)
      readA(st, 1);
      if (pre2) dmaB(0, st, kt + 2);
      NR_PHASE_SYNC_MMA(1, 1, fb1)
      if (pre2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (pre2) dmaB(1, st, kt + 2);
      __builtin_amdgcn_s_setprio(1);
      mma(1, 0, fb0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
    }
    if (wmu == 0) __builtin_amdgcn_s_barrier();  // re-align the groups: every stage read is retired
    const int64_t n0 = tn0, m0 = tm0;
    const int tn = t + t_step;
    const bool more = tn < t_end;
    // everything the epilogue reads from memory is loaded BEFORE the next
    // tile's DMAs: a later load's wait would also wait for the (older) DMAs
    float b16[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) b16[ni] = bias[n0 + wn * 64 + 16 * ni + (lane & 15)];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (more) {  // next tile's operands fly while this tile's epilogue runs
      setup(tn);
      prologue();
    }
    epi16_store<EPI, TO>(acc, slab, lane, wm, wn, m0, n0, M, N, b16, R, ldr, C, ldc, ea);
    if (!more) break;
    drain_all = m0 + G2BM > M;  // ragged tile: some stores were skipped
    t = tn;
  }
#undef NR_PHASE_SYNC_MMA
}

template <typename TO>
static int launch_gemm256_pp(int epi, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                             const void* W, int64_t ldw, const float* bias, const void* R, int64_t ldr,
                             void* C, int64_t ldc, const EpiArgs& ea, hipStream_t s) {
  const int tiles_n = (int)(N / G2BN);
  const int64_t tiles = (int64_t)tiles_n * ((M + G2BM - 1) / G2BM);
  if (tiles > (1ll << 30)) {
    set_error("nr_gemm: too many tiles");
    return NR_ERR_UNSUPPORTED;
  }
  const int nt = (int)tiles;
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    hipDeviceProp_t prop;
    n_cu = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
               ? prop.multiProcessorCount : 256;
    n_cu = n_cu / 8 * 8;
    if (n_cu < 8) n_cu = 8;
  }
  const dim3 grid((unsigned)(nt < n_cu ? nt : n_cu));
  const __bf16* a = (const __bf16*)A;
  const __bf16* w = (const __bf16*)W;
  const TO* r = (const TO*)R;
  TO* c = (TO*)C;
#define NR_PP(E) hipLaunchKernelGGL((gemm256pp_kernel<E, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea, tiles_n, nt)
  switch (epi) {
    case NR_EPI_NONE: NR_PP(NR_EPI_NONE); break;
    case NR_EPI_RELU: NR_PP(NR_EPI_RELU); break;
    case NR_EPI_EXP: NR_PP(NR_EPI_EXP); break;
    case NR_EPI_GEGLU: NR_PP(NR_EPI_GEGLU); break;
    case NR_EPI_RESADD: NR_PP(NR_EPI_RESADD); break;
    case NR_EPI_GELU: NR_PP(NR_EPI_GELU); break;
    case NR_EPI_RELU_DROPOUT: NR_PP(NR_EPI_RELU_DROPOUT); break;
    case NR_EPI_DRELU: NR_PP(NR_EPI_DRELU); break;
    case NR_EPI_SOFTMAX64: NR_PP(NR_EPI_SOFTMAX64); break;
    default: set_error("nr_gemm: bad epilogue %d", epi); return NR_ERR_INVALID;
  }
#undef NR_PP
  NR_CHECK_LAUNCH("nr_gemm");
  return NR_OK;
}

template <typename TI, typename TO>
static int launch_gemm256_v1(int epi, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                          const void* W, int64_t ldw, const float* bias, const void* R, int64_t ldr,
                          void* C, int64_t ldc, const EpiArgs& ea, hipStream_t s) {
  dim3 grid((unsigned)(N / G2BN), (unsigned)((M + G2BM - 1) / G2BM));
  const TI* a = (const TI*)A;
  const TI* w = (const TI*)W;
  const TO* r = (const TO*)R;
  TO* c = (TO*)C;
  switch (epi) {
    case NR_EPI_NONE: hipLaunchKernelGGL((gemm256_kernel<TI, NR_EPI_NONE, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RELU: hipLaunchKernelGGL((gemm256_kernel<TI, NR_EPI_RELU, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_EXP: hipLaunchKernelGGL((gemm256_kernel<TI, NR_EPI_EXP, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_GEGLU: hipLaunchKernelGGL((gemm256_kernel<TI, NR_EPI_GEGLU, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RESADD: hipLaunchKernelGGL((gemm256_kernel<TI, NR_EPI_RESADD, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_GELU: hipLaunchKernelGGL((gemm256_kernel<TI, NR_EPI_GELU, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_RELU_DROPOUT: hipLaunchKernelGGL((gemm256_kernel<TI, NR_EPI_RELU_DROPOUT, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_DRELU: hipLaunchKernelGGL((gemm256_kernel<TI, NR_EPI_DRELU, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    case NR_EPI_SOFTMAX64: hipLaunchKernelGGL((gemm256_kernel<TI, NR_EPI_SOFTMAX64, TO>), grid, dim3(512), 0, s, M, N, K, a, lda, w, ldw, bias, r, ldr, c, ldc, ea); break;
    default: set_error("nr_gemm: bad epilogue %d", epi); return NR_ERR_INVALID;
  }
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

template <typename TI, typename TO>
static int launch_gemm256(int epi, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                          const void* W, int64_t ldw, const float* bias, const void* R, int64_t ldr,
                          void* C, int64_t ldc, const EpiArgs& ea, hipStream_t s) {
  static const bool v1 = getenv("NR_GEMM_V1") != nullptr;  // A/B switch: the 2-stage glds kernel
  // bf16 default: 16x16x32 MFMA tiles (5-8 % faster than 32x32x16 on the pooler shapes,
  // profiles/round1/s2/gemm_mf16_vs_mf32.txt); NR_GEMM_MF32=1 selects the 32x32x16 tiles
  static const bool mf16 = getenv("NR_GEMM_MF32") == nullptr;
  if (v1) return launch_gemm256_v1<TI, TO>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, ea, s);
  // persistent variant: opt-in (NR_GEMM_PERSIST=1) until its register pressure is fixed: its
  // spill reloads in the epilogue wait on the next tile's DMAs
  static const bool persist = getenv("NR_GEMM_PERSIST") != nullptr;
  // tile order (tile_of): NR_GEMM_GROUP_M overrides the default M-tile group
  static const int group_m = getenv("NR_GEMM_GROUP_M") ? atoi(getenv("NR_GEMM_GROUP_M")) : 4;
  EpiArgs eg = ea;
  eg.group_m = group_m;
  if constexpr (sizeof(TI) == 2) {
    if (mf16 && persist) return launch_gemm256_pp<TO>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, eg, s);
    if (mf16) return launch_gemm256_p16<TI, TO>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, eg, s);
  }
  return launch_gemm256_p<TI, TO>(epi, M, N, K, A, lda, W, ldw, bias, R, ldr, C, ldc, eg, s);
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
  NR_CHECK_ARG((epi != NR_EPI_RESADD && epi != NR_EPI_DRELU) || R, "nr_gemm: RESADD/DRELU need R");
  NR_CHECK_ARG(epi >= NR_EPI_NONE && epi <= NR_EPI_SOFTMAX64, "nr_gemm: bad epilogue %d", epi);
  const int64_t e16 = dtype_in == NR_F32 ? 4 : 8;  // elements per 16 B
  NR_CHECK_ARG(lda >= K && ldw >= K && lda % e16 == 0 && ldw % e16 == 0 &&
                   ((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0,
               "nr_gemm: A/W must be 16-byte aligned with 16-byte row strides");
  const int64_t ncols = epi == NR_EPI_GEGLU ? N / 2 : N;
  NR_CHECK_ARG(ldc >= ncols, "nr_gemm: ldc too small");
  NR_CHECK_ARG((M + GBM - 1) / GBM <= 65535, "nr_gemm: M too large (> 8.3M rows)");
  // 256x256 glds kernel when the shape allows (every pooler GEMM); the
  // 128x128 register-staged kernel covers N % 256 != 0 and unaligned outputs.
  static const bool force_small = getenv("NR_GEMM_SMALL_TILE") != nullptr;  // A/B switch for profiling
  const int64_t vo = dtype_out == NR_F32 ? 4 : 8;  // the LDS-staged epilogue stores 16 B per lane
  const bool aligned_out = ((uintptr_t)C & 15) == 0 && ldc % vo == 0 &&
                           ((epi != NR_EPI_RESADD && epi != NR_EPI_DRELU) || (((uintptr_t)R & 15) == 0 && ldr % vo == 0));
  const bool big = (N % G2BN == 0) && aligned_out && !force_small;
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
  const double t = (double)p * 4294967296.0;
  const uint32_t thr = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  return nr::gemm_dispatch_ex(dtype_in, dtype_out, NR_EPI_RELU_DROPOUT, M, N, K, A, lda, W, ldw, bias, nullptr, 0,
                              C, ldc, nr::EpiArgs{seed, thr, 1.0f / (1.0f - p)}, (hipStream_t)stream);
}

extern "C" int nr_gemm_drelu(int dtype_in, int dtype_out, int64_t M, int64_t N, int64_t K, const void* A,
                             int64_t lda, const void* W, int64_t ldw, const void* Y, int64_t ldy, void* C,
                             int64_t ldc, float scale, void* stream) {
  nr::clear_error();
  return nr::gemm_dispatch_ex(dtype_in, dtype_out, NR_EPI_DRELU, M, N, K, A, lda, W, ldw, nullptr, Y, ldy, C, ldc,
                              nr::EpiArgs{0, 0, scale}, (hipStream_t)stream);
}

extern "C" int nr_gemm(int dtype_in, int dtype_out, int epilogue, int64_t M, int64_t N, int64_t K,
                       const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
                       const void* R, int64_t ldr, void* C, int64_t ldc, void* stream) {
  nr::clear_error();
  return nr::gemm_dispatch(dtype_in, dtype_out, epilogue, M, N, K, A, lda, W, ldw, bias, R, ldr, C,
                           ldc, (hipStream_t)stream);
}

extern "C" int nr_gemm_grouped(int dtype_in, int dtype_out, int n, const int64_t* M, const int64_t* N,
                               const int64_t* K, const void* const* A, const int64_t* lda, const void* const* W,
                               const int64_t* ldw, void* const* C, const int64_t* ldc, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(dtype_in == NR_BF16 || dtype_in == NR_F32, "nr_gemm_grouped: bad dtype_in %d", dtype_in);
  NR_CHECK_ARG(dtype_out == NR_F32 || dtype_out == NR_BF16, "nr_gemm_grouped: bad dtype_out %d", dtype_out);
  NR_CHECK_ARG(n >= 1 && n <= NR_GEMM_MAX_GROUP, "nr_gemm_grouped: n=%d outside [1, %d]", n, NR_GEMM_MAX_GROUP);
  NR_CHECK_ARG(M && N && K && A && lda && W && ldw && C && ldc, "nr_gemm_grouped: null array");
  nr::GemmGroup g{};
  g.n = 0;
  int64_t tiles = 0;
  const int64_t vo = dtype_out == NR_F32 ? 4 : 8;
  for (int i = 0; i < n; ++i) {
    const int64_t bk = dtype_in == NR_F32 ? 32 : 64, e16 = dtype_in == NR_F32 ? 4 : 8;
    NR_CHECK_ARG(M[i] >= 0 && N[i] > 0 && K[i] > 0 && N[i] % nr::G2BN == 0 && K[i] % bk == 0,
                 "nr_gemm_grouped: problem %d bad shape M=%lld N=%lld K=%lld (need N %% 256, K %% 64 bf16 / 32 f32)", i,
                 (long long)M[i], (long long)N[i], (long long)K[i]);
    if (M[i] == 0) continue;  // empty problem: no operand is read (torch gives a null data pointer)
    NR_CHECK_ARG(A[i] && W[i] && C[i], "nr_gemm_grouped: problem %d null operand", i);
    NR_CHECK_ARG(lda[i] >= K[i] && ldw[i] >= K[i] && lda[i] % e16 == 0 && ldw[i] % e16 == 0 && ldc[i] >= N[i] &&
                     ldc[i] % vo == 0 && ((uintptr_t)A[i] & 15) == 0 && ((uintptr_t)W[i] & 15) == 0 &&
                     ((uintptr_t)C[i] & 15) == 0,
                 "nr_gemm_grouped: problem %d operands must be 16-byte aligned with 16-byte row strides", i);
    const int j = g.n++;
    g.M[j] = M[i]; g.N[j] = N[i]; g.K[j] = K[i];
    g.A[j] = A[i]; g.W[j] = W[i]; g.C[j] = C[i];
    g.lda[j] = lda[i]; g.ldw[j] = ldw[i]; g.ldc[j] = ldc[i];
    g.ntn[j] = (int)(N[i] / nr::G2BN);
    tiles += ((M[i] + nr::G2BM - 1) / nr::G2BM) * g.ntn[j];
    NR_CHECK_ARG(tiles <= 0x7fffffff, "nr_gemm_grouped: too many tiles");
    g.tile_end[j] = (int)tiles;
  }
  if (g.n == 0) return NR_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype_in == NR_F32 && dtype_out == NR_F32)
    hipLaunchKernelGGL((nr::gemm256p_group_kernel<float, float, false>), dim3((unsigned)tiles), dim3(512), 0, s, g);
  else if (dtype_in == NR_F32)
    hipLaunchKernelGGL((nr::gemm256p_group_kernel<float, __bf16, false>), dim3((unsigned)tiles), dim3(512), 0, s, g);
  else if (dtype_out == NR_F32)
    hipLaunchKernelGGL((nr::gemm256p_group_kernel<__bf16, float, true>), dim3((unsigned)tiles), dim3(512), 0, s, g);
  else
    hipLaunchKernelGGL((nr::gemm256p_group_kernel<__bf16, __bf16, true>), dim3((unsigned)tiles), dim3(512), 0, s, g);
  NR_CHECK_LAUNCH("nr_gemm_grouped");
  return NR_OK;
}

#if NR_GEMM_STAMPS
extern "C" int nr_debug_gemm_stamps(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(nr::g_gemm_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif
