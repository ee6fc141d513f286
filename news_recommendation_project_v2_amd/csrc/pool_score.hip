// Fused segmented history pooling + candidate cosine scoring (gfx950).
//
// Replaces, for every impression i of the eval set:
//   get_final_attention_eval   data_model_helper.py:112-131  (padded batches
//       through FinalAttention.forward modeling_utils.py:224-228, or
//       LatentAttentionModel.forward latent_attention.py:165-170)
//   get_cos_sim_scores loop    data_model_helper.py:199-230  (F.cosine_similarity)
//
// The per-item pooler transform is computed once per unique news by the GEMM
// chain (gemm.hip); this kernel only gathers table rows:
//   FINAL : u = sum_j x_j*p_j / (sum_j p_j + 1e-10)     (p = exp(w), per dim)
//   LATENT: u = normalize(sum_j h_j / h_i, eps 1e-12)
//   MEAN  : u = sum_j h_j / h_i            (average_pool, modeling_utils.py:55-59)
//   score_c = (u . e_c) / max(|u|, 1e-8) / max(|e_c|, 1e-8)
//
// Work decomposition: one wave (64 lanes) per impression, 4 impressions per
// 256-thread workgroup.  A table row is D=1024 elements = 16 per lane, read as
// 16-byte lane loads (1 KiB per wave instruction, fully coalesced within the
// row).  Row indices are loaded 64 at a time (one per lane) and broadcast with
// v_readlane, so row addresses are wave-uniform.  Several rows are kept in
// flight per wave (history: 2-4 rows, candidates: 4 rows) to cover gather
// latency; candidate dot products are reduced across the wave 4 at a time with
// a transpose-reduce (7 cross-lane steps for 4 dots instead of 24).
#include "nr_common.h"

namespace nr {

template <typename T, int DIM>
struct RowFmt {
  static constexpr int VEC = 16 / (int)sizeof(T);  // elements per 16-B load
  static constexpr int NL = DIM / (64 * VEC);       // 16-B loads per lane per row
  static constexpr int EPL = DIM / 64;              // elements per lane
  static_assert(DIM % (64 * VEC) == 0, "DIM must be a multiple of 64*VEC");
};

template <typename T, int DIM>
__device__ __forceinline__ void load_row(const T* __restrict__ row, int lane,
                                         uint4 (&r)[RowFmt<T, DIM>::NL]) {
  const uint4* p = reinterpret_cast<const uint4*>(row) + lane;
#pragma unroll
  for (int j = 0; j < RowFmt<T, DIM>::NL; ++j) r[j] = p[j * 64];
}

template <typename T, int DIM>
__device__ __forceinline__ void unpack_row(const uint4 (&r)[RowFmt<T, DIM>::NL],
                                           float (&v)[RowFmt<T, DIM>::EPL]) {
  constexpr int NL = RowFmt<T, DIM>::NL;
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      v[4 * j + 0] = __uint_as_float(r[j].x);
      v[4 * j + 1] = __uint_as_float(r[j].y);
      v[4 * j + 2] = __uint_as_float(r[j].z);
      v[4 * j + 3] = __uint_as_float(r[j].w);
    }
  } else {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      v[8 * j + 0] = bf16_lo(r[j].x);
      v[8 * j + 1] = bf16_hi(r[j].x);
      v[8 * j + 2] = bf16_lo(r[j].y);
      v[8 * j + 3] = bf16_hi(r[j].y);
      v[8 * j + 4] = bf16_lo(r[j].z);
      v[8 * j + 5] = bf16_hi(r[j].z);
      v[8 * j + 6] = bf16_lo(r[j].w);
      v[8 * j + 7] = bf16_hi(r[j].w);
    }
  }
}

// Element index (within the row) of lane-local element i.
template <typename T, int DIM>
__device__ __forceinline__ int elem_pos(int i, int lane) {
  constexpr int VEC = RowFmt<T, DIM>::VEC;
  return (i / VEC) * (64 * VEC) + lane * VEC + (i % VEC);
}

template <typename T, int POOL>
struct PoolCfg;
// rows of history kept in flight per wave: ~16 x 16-B loads per lane
template <> struct PoolCfg<float, NR_POOL_FINAL> { static constexpr int R = 2; };
template <> struct PoolCfg<float, NR_POOL_LATENT> { static constexpr int R = 4; };
template <> struct PoolCfg<__bf16, NR_POOL_FINAL> { static constexpr int R = 4; };
template <> struct PoolCfg<__bf16, NR_POOL_LATENT> { static constexpr int R = 8; };
template <> struct PoolCfg<float, NR_POOL_MEAN> { static constexpr int R = 4; };
template <> struct PoolCfg<__bf16, NR_POOL_MEAN> { static constexpr int R = 8; };

// transpose-reduce of 4 per-lane partial dots; returns the total of dot q in
// lane 16*q (and its 15 neighbours).
__device__ __forceinline__ float reduce4(const float (&d)[4], int lane) {
  const bool hi = lane & 32;
  const float s0 = hi ? d[0] : d[2], s1 = hi ? d[1] : d[3];
  const float k0 = hi ? d[2] : d[0], k1 = hi ? d[3] : d[1];
  const float a0 = k0 + __shfl_xor(s0, 32, 64);
  const float a1 = k1 + __shfl_xor(s1, 32, 64);
  const bool m16 = lane & 16;
  float b = (m16 ? a1 : a0) + __shfl_xor(m16 ? a0 : a1, 16, 64);
  b += __shfl_xor(b, 8, 64);
  b += __shfl_xor(b, 4, 64);
  b += __shfl_xor(b, 2, 64);
  b += __shfl_xor(b, 1, 64);
  return b;
}

// FROM_USERS: the user vector of impression i is row uidx[i] of a table of
// user vectors this kernel wrote earlier (users output of a pooling-only
// launch over the distinct histories), instead of its own history gather; the
// candidate pass is the same code, so the scores are bit-identical.
template <typename T, int POOL, int DIM, bool FROM_USERS = false>
__global__ __launch_bounds__(256) void pool_score_kernel(
    const T* __restrict__ htab, int64_t hld, const T* __restrict__ ctab, int64_t cld,
    const float* __restrict__ cinv, const int32_t* __restrict__ hidx,
    const int64_t* __restrict__ hoff, const int32_t* __restrict__ cidx,
    const int64_t* __restrict__ coff, int64_t n_imp, float* __restrict__ scores,
    float* __restrict__ users, const int32_t* __restrict__ uidx) {
  using F = RowFmt<T, DIM>;
  constexpr int NL = F::NL, EPL = F::EPL;
  constexpr int R = PoolCfg<T, POOL>::R;
  constexpr int G = 4;

  const int lane = threadIdx.x & 63;
  const int64_t imp = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (imp >= n_imp) return;  // wave-uniform

  float u[EPL];
  if constexpr (FROM_USERS) {
    const float* ur = users + (int64_t)uidx[imp] * DIM;
#pragma unroll
    for (int i = 0; i < EPL; ++i) u[i] = ur[elem_pos<T, DIM>(i, lane)];
  } else {
  float acc[EPL];
  float den[EPL];
#pragma unroll
  for (int i = 0; i < EPL; ++i) { acc[i] = 0.f; den[i] = 0.f; }

  // ---------------- history pooling ----------------
  const int64_t h0 = hoff[imp], h1 = hoff[imp + 1];
  for (int64_t base = h0; base < h1; base += 64) {
    const int cnt = (int)min((int64_t)64, h1 - base);
    // hidx == nullptr: the segment's rows are consecutive table rows (token pooling)
    const int myidx = lane < cnt ? (hidx ? hidx[base + lane] : (int)(base + lane)) : 0;
    int r = 0;
    for (; r + R <= cnt; r += R) {
      uint4 bx[R][NL];
      uint4 bp[(POOL == NR_POOL_FINAL) ? R : 1][NL];
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const int row = __builtin_amdgcn_readlane(myidx, r + q);
        const T* p = htab + (int64_t)row * hld;
        load_row<T, DIM>(p, lane, bx[q]);
        if constexpr (POOL == NR_POOL_FINAL) load_row<T, DIM>(p + DIM, lane, bp[q]);
      }
#pragma unroll
      for (int q = 0; q < R; ++q) {
        float x[EPL];
        unpack_row<T, DIM>(bx[q], x);
        if constexpr (POOL == NR_POOL_FINAL) {
          float pw[EPL];
          unpack_row<T, DIM>(bp[q], pw);
#pragma unroll
          for (int i = 0; i < EPL; ++i) { acc[i] = fmaf(x[i], pw[i], acc[i]); den[i] += pw[i]; }
        } else {
#pragma unroll
          for (int i = 0; i < EPL; ++i) acc[i] += x[i];
        }
      }
    }
    for (; r < cnt; ++r) {
      const int row = __builtin_amdgcn_readlane(myidx, r);
      const T* p = htab + (int64_t)row * hld;
      uint4 bx[NL];
      load_row<T, DIM>(p, lane, bx);
      float x[EPL];
      unpack_row<T, DIM>(bx, x);
      if constexpr (POOL == NR_POOL_FINAL) {
        uint4 bp[NL];
        load_row<T, DIM>(p + DIM, lane, bp);
        float pw[EPL];
        unpack_row<T, DIM>(bp, pw);
#pragma unroll
        for (int i = 0; i < EPL; ++i) { acc[i] = fmaf(x[i], pw[i], acc[i]); den[i] += pw[i]; }
      } else {
#pragma unroll
        for (int i = 0; i < EPL; ++i) acc[i] += x[i];
      }
    }
  }

  // ---------------- user vector ----------------
  if constexpr (POOL == NR_POOL_FINAL) {
    // modeling_utils.py:224-228: w = exp(w)*m; w /= (sum w + 1e-10); sum x*w
#pragma unroll
    for (int i = 0; i < EPL; ++i) u[i] = acc[i] / (den[i] + 1e-10f);
  } else if constexpr (POOL == NR_POOL_MEAN) {
    const float d = (float)(h1 - h0);
#pragma unroll
    for (int i = 0; i < EPL; ++i) u[i] = acc[i] / d;
  } else {
    // latent_attention.py:166-170: s / d, then F.normalize(p=2, eps=1e-12)
    const float d = (float)(h1 - h0);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < EPL; ++i) { u[i] = acc[i] / d; ss = fmaf(u[i], u[i], ss); }
    const float nrm = sqrtf(wave_sum(ss));
    const float den1 = fmaxf(nrm, 1e-12f);
#pragma unroll
    for (int i = 0; i < EPL; ++i) u[i] = u[i] / den1;
  }
  if (users != nullptr) {
    float* ur = users + imp * DIM;
#pragma unroll
    for (int i = 0; i < EPL; ++i) ur[elem_pos<T, DIM>(i, lane)] = u[i];
  }
  }  // !FROM_USERS
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) ss = fmaf(u[i], u[i], ss);
  const float inv_u = 1.0f / fmaxf(sqrtf(wave_sum(ss)), 1e-8f);

  // ---------------- candidate scoring ----------------
  if (coff == nullptr) return;  // pooling only
  const int64_t c0 = coff[imp], c1 = coff[imp + 1];
  for (int64_t base = c0; base < c1; base += 64) {
    const int cnt = (int)min((int64_t)64, c1 - base);
    const int myidx = lane < cnt ? cidx[base + lane] : 0;
    const float myinv = lane < cnt ? cinv[myidx] : 0.f;
    float mydot = 0.f;
    for (int r = 0; r < cnt; r += G) {
      uint4 bc[G][NL];
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const int rr = min(r + q, cnt - 1);
        const int row = __builtin_amdgcn_readlane(myidx, rr);
        load_row<T, DIM>(ctab + (int64_t)row * cld, lane, bc[q]);
      }
      float d[G];
#pragma unroll
      for (int q = 0; q < G; ++q) {
        float e[EPL];
        unpack_row<T, DIM>(bc[q], e);
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < EPL; ++i) s = fmaf(u[i], e[i], s);
        d[q] = s;
      }
      const float b = reduce4(d, lane);
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const float t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b), 16 * q));
        if (lane == r + q) mydot = t;
      }
    }
    if (lane < cnt) scores[base + lane] = mydot * inv_u * myinv;
  }
}

template <typename T, int POOL, bool FROM_USERS = false>
static int launch_pool_score(const void* ht, int64_t hld, const void* ct, int64_t cld,
                             const float* cinv, const int32_t* hidx, const int64_t* hoff,
                             const int32_t* cidx, const int64_t* coff, int64_t n_imp,
                             float* scores, float* users, hipStream_t s, const int32_t* uidx = nullptr) {
  const int64_t blocks = (n_imp + 3) / 4;
  hipLaunchKernelGGL((pool_score_kernel<T, POOL, 1024, FROM_USERS>), dim3((unsigned)blocks), dim3(256), 0, s,
                     (const T*)ht, hld, (const T*)ct, cld, cinv, hidx, hoff, cidx, coff, n_imp,
                     scores, users, uidx);
  NR_CHECK_LAUNCH("nr_pool_score");
  return NR_OK;
}

// Pooling only (no candidates) of consecutive rows: segment i = table rows
// off[i] .. off[i+1]-1, u written to users [n_seg][1024] f32.
int pool_rows_dispatch(int pooler, int dtype, const void* table, int64_t ld, const int64_t* off, int64_t n_seg,
                       float* users, hipStream_t s) {
  if (n_seg == 0) return NR_OK;
  if (dtype == NR_F32) {
    if (pooler == NR_POOL_MEAN)
      return launch_pool_score<float, NR_POOL_MEAN>(table, ld, table, ld, nullptr, nullptr, off, nullptr, nullptr, n_seg, nullptr, users, s);
    return launch_pool_score<float, NR_POOL_LATENT>(table, ld, table, ld, nullptr, nullptr, off, nullptr, nullptr, n_seg, nullptr, users, s);
  }
  if (pooler == NR_POOL_MEAN)
    return launch_pool_score<__bf16, NR_POOL_MEAN>(table, ld, table, ld, nullptr, nullptr, off, nullptr, nullptr, n_seg, nullptr, users, s);
  return launch_pool_score<__bf16, NR_POOL_LATENT>(table, ld, table, ld, nullptr, nullptr, off, nullptr, nullptr, n_seg, nullptr, users, s);
}

}  // namespace nr

extern "C" int nr_pool_score(int pooler, int dtype, int64_t dim, const void* hist_table,
                             int64_t hist_ld, const void* cand_table, int64_t cand_ld,
                             const float* cand_inv_norm, const int32_t* hist_idx,
                             const int64_t* hist_off, const int32_t* cand_idx,
                             const int64_t* cand_off, int64_t n_imp, float* scores,
                             float* users, void* stream) {
  nr::clear_error();
  if (dim != 1024) {
    nr::set_error("nr_pool_score: dim %lld unsupported (1024 only)", (long long)dim);
    return NR_ERR_UNSUPPORTED;
  }
  NR_CHECK_ARG(pooler == NR_POOL_FINAL || pooler == NR_POOL_LATENT || pooler == NR_POOL_MEAN,
               "nr_pool_score: bad pooler %d", pooler);
  NR_CHECK_ARG(dtype == NR_F32 || dtype == NR_BF16, "nr_pool_score: bad dtype %d", dtype);
  NR_CHECK_ARG(n_imp >= 0, "nr_pool_score: n_imp < 0");
  if (n_imp == 0) return NR_OK;
  const bool score = cand_off != nullptr;
  NR_CHECK_ARG(hist_table && hist_off && (score || users), "nr_pool_score: null pointer");
  NR_CHECK_ARG(!score || (cand_table && cand_inv_norm && cand_idx && scores), "nr_pool_score: null candidate pointer");
  NR_CHECK_DEVICE("nr_pool_score", hist_table, cand_table, cand_inv_norm, hist_idx, hist_off, cand_idx, cand_off,
                  scores, users);
  if (!score) {
    cand_table = hist_table;
    cand_ld = hist_ld;
  }
  const int64_t min_hld = pooler == NR_POOL_FINAL ? 2 * dim : dim;
  NR_CHECK_ARG(hist_ld >= min_hld && cand_ld >= dim, "nr_pool_score: leading dimension too small");
  const int64_t align = dtype == NR_F32 ? 4 : 8;
  NR_CHECK_ARG(hist_ld % align == 0 && cand_ld % align == 0 &&
                   ((uintptr_t)hist_table & 15) == 0 && ((uintptr_t)cand_table & 15) == 0,
               "nr_pool_score: tables must be 16-byte aligned with 16-byte row strides");
  hipStream_t s = (hipStream_t)stream;
  if (pooler == NR_POOL_MEAN) {
    if (dtype == NR_F32)
      return nr::launch_pool_score<float, NR_POOL_MEAN>(hist_table, hist_ld, cand_table, cand_ld, cand_inv_norm, hist_idx, hist_off, cand_idx, cand_off, n_imp, scores, users, s);
    return nr::launch_pool_score<__bf16, NR_POOL_MEAN>(hist_table, hist_ld, cand_table, cand_ld, cand_inv_norm, hist_idx, hist_off, cand_idx, cand_off, n_imp, scores, users, s);
  }
  if (dtype == NR_F32) {
    if (pooler == NR_POOL_FINAL)
      return nr::launch_pool_score<float, NR_POOL_FINAL>(hist_table, hist_ld, cand_table, cand_ld, cand_inv_norm, hist_idx, hist_off, cand_idx, cand_off, n_imp, scores, users, s);
    return nr::launch_pool_score<float, NR_POOL_LATENT>(hist_table, hist_ld, cand_table, cand_ld, cand_inv_norm, hist_idx, hist_off, cand_idx, cand_off, n_imp, scores, users, s);
  }
  if (pooler == NR_POOL_FINAL)
    return nr::launch_pool_score<__bf16, NR_POOL_FINAL>(hist_table, hist_ld, cand_table, cand_ld, cand_inv_norm, hist_idx, hist_off, cand_idx, cand_off, n_imp, scores, users, s);
  return nr::launch_pool_score<__bf16, NR_POOL_LATENT>(hist_table, hist_ld, cand_table, cand_ld, cand_inv_norm, hist_idx, hist_off, cand_idx, cand_off, n_imp, scores, users, s);
}

extern "C" int nr_score_users(int dtype, int64_t dim, const float* users, const int32_t* user_idx,
                              const void* cand_table, int64_t cand_ld, const float* cand_inv_norm,
                              const int32_t* cand_idx, const int64_t* cand_off, int64_t n_imp, float* scores,
                              void* stream) {
  nr::clear_error();
  if (dim != 1024) {
    nr::set_error("nr_score_users: dim %lld unsupported (1024 only)", (long long)dim);
    return NR_ERR_UNSUPPORTED;
  }
  NR_CHECK_ARG(dtype == NR_F32 || dtype == NR_BF16, "nr_score_users: bad dtype %d", dtype);
  NR_CHECK_ARG(n_imp >= 0, "nr_score_users: n_imp < 0");
  if (n_imp == 0) return NR_OK;
  NR_CHECK_ARG(users && user_idx && cand_table && cand_inv_norm && cand_idx && cand_off && scores,
               "nr_score_users: null pointer");
  NR_CHECK_DEVICE("nr_score_users", users, user_idx, cand_table, cand_inv_norm, cand_idx, cand_off, scores);
  NR_CHECK_ARG(cand_ld >= dim && cand_ld % (dtype == NR_F32 ? 4 : 8) == 0 && ((uintptr_t)cand_table & 15) == 0,
               "nr_score_users: cand_table must be 16-byte aligned with 16-byte row strides");
  hipStream_t s = (hipStream_t)stream;
  // the pooler only shaped the stored user vectors; the scoring pass is pooler-independent
  if (dtype == NR_F32)
    return nr::launch_pool_score<float, NR_POOL_MEAN, true>(nullptr, 0, cand_table, cand_ld, cand_inv_norm, nullptr,
                                                            nullptr, cand_idx, cand_off, n_imp, scores,
                                                            const_cast<float*>(users), s, user_idx);
  return nr::launch_pool_score<__bf16, NR_POOL_MEAN, true>(nullptr, 0, cand_table, cand_ld, cand_inv_norm, nullptr,
                                                           nullptr, cand_idx, cand_off, n_imp, scores,
                                                           const_cast<float*>(users), s, user_idx);
}
