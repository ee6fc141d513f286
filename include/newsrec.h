/*
 * newsrec.h — C-ABI of libnewsrec_hip.so, the MI355X (gfx950) kernels behind
 * the MIND embed -> pool -> score hot path.
 *
 * The reference (AhmedFahim-git/news_recommendation_project_v2) has no native
 * code and no FFI: its boundary is the Python API of src/news_rec_utils
 * (SURVEY.md §8(b)).  These entry points replace the torch ops that API calls,
 * and are bound from Python with ctypes by
 * news_recommendation_project_v2_amd/_lib.py (see INTEGRATION.md for the
 * binding a maintainer would add to the reference).
 *
 * Conventions
 *  - Every device buffer is allocated and freed by the caller (PyTorch); the
 *    library never frees caller memory.  Scratch is an explicit workspace.
 *  - All calls enqueue asynchronously on `stream` (a hipStream_t passed as
 *    void*; NULL = the legacy default stream) and never synchronise, so they
 *    are graph-capturable.
 *  - Return NR_OK (0) or a negative code; nr_last_error() returns the
 *    thread-local message of the last failure.  No exception crosses the ABI.
 *  - Reentrant: host threads may call concurrently, each on its own stream
 *    (scratch is the caller's workspace; error strings and residency caches
 *    are thread-local; the two process-wide knobs below are atomics).  A
 *    row's output bits do not depend on how the rows were cut into calls.
 *  - Matrices are row-major with explicit leading dimensions in ELEMENTS.
 *    Linear weights use torch's nn.Linear layout W[out_features][in_features],
 *    so GEMMs compute C = A · Wᵀ.
 */
#ifndef NEWSREC_H
#define NEWSREC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NR_OK 0
#define NR_ERR_INVALID -1     /* bad argument / shape */
#define NR_ERR_HIP -2         /* HIP runtime or launch failure */
#define NR_ERR_UNSUPPORTED -3 /* valid but not implemented (e.g. dim) */
#define NR_ERR_TIMEOUT -4     /* a collective did not complete within its deadline */

/* element types */
#define NR_F32 0
#define NR_BF16 1
#define NR_F16 2 /* input-only, nr_gather_layernorm (token states are stored fp16) */

/* history poolers */
#define NR_POOL_FINAL 0  /* FinalAttention additive per-dim softmax pooler */
#define NR_POOL_LATENT 1 /* LatentAttentionModel masked mean + L2 normalize */
#define NR_POOL_MEAN 2   /* masked mean only (average_pool, modeling_utils.py:55-59) */
#define NR_POOL_NONE -1  /* nr_encoder_forward: no pooling (per-token hidden states only) */

/* GEMM epilogues (applied to acc = A·Wᵀ) */
#define NR_EPI_NONE 0   /* C = acc + bias                                   */
#define NR_EPI_RELU 1   /* C = relu(acc + bias)                             */
#define NR_EPI_EXP 2    /* C = exp(acc + bias)                              */
#define NR_EPI_GEGLU 3  /* W rows interleaved in 32-row (a, g) blocks:
                           C[:, j] = (a_j + ba_j) * gelu_erf(g_j + bg_j);
                           C has N/2 columns                               */
#define NR_EPI_RESADD 4 /* C = acc + bias + R                               */
#define NR_EPI_GELU 5   /* C = gelu_erf(acc + bias)                         */
#define NR_EPI_RELU_DROPOUT 6 /* C = relu(acc + bias) * keep / (1 - p), training
                                 forward only: use nr_gemm_relu_dropout      */
#define NR_EPI_DRELU 7  /* C = R > 0 ? acc * scale : 0 (backward of relu+dropout
                           given its forward output R): nr_gemm_drelu       */
#define NR_EPI_SOFTMAX64 8 /* C = softmax over each aligned run of 64 columns of
                           (acc + bias): SDPA's softmax over the 64 latents of
                           latent_attention.py:72 fused into the score GEMM
                           (needs N % 256 == 0, 16-byte aligned C rows)      */
#define NR_EPI_SOFTMAX64_BWD 9 /* C = R * (acc - sum over the aligned run of 64 columns
                           of R * acc): the backward of NR_EPI_SOFTMAX64 given its
                           output R = P and acc = dP (latent training; bf16 in /
                           out on the persistent kernel only)               */

/* Library version (major*100 + minor). */
int nr_version(void);

/* Hash of the sources the library was built from (16 hex digits: sha256 of
 * csrc/{capi,gemm,pool_score,rowops,rank,encoder,train,metrics,comm,latent_train}.hip,
 * csrc/nr_common.h and this header, concatenated in that order); the Python
 * loader refuses a library whose hash differs from the tree it sits in. */
const char* nr_build_hash(void);

/* Select the HIP device for subsequent calls on this host thread and load the
 * code object once per device.  Replaces the implicit `.to(DEVICE)` of
 * config.py:19 for the library's own state. */
int nr_init(int device);

/* Workgroups of the persistent bf16 GEMM launches (one per CU by default).
 * For callers that run the transform on a CU-masked stream beside other
 * work (hipExtStreamCreateWithCUMask): set it to the stream's CU count.
 * n = 0 restores the default; otherwise n must be a positive multiple of 8
 * (the kernel maps blockIdx % 8 to an XCD).  Process-wide (an atomic): a
 * launch on another thread uses whichever value it reads. */
int nr_set_persistent_workgroups(int n);

/* The current budget (0 = the default, one workgroup per CU), so a caller can
 * restore what it found. */
int nr_persistent_workgroups(void);

/* Half-tile tail of the persistent bf16 GEMM (on by default).  When the
 * output tiles leave a last partial round of at most half the grid, those
 * tiles run as 128-row halves, one per workgroup, so the round takes about
 * half a tile's time.  A row's bits are the same either way (same K chain and
 * epilogue per element): the switch exists for A/B timing.  Process-wide. */
int nr_set_gemm_half_tail(int on);

/* Thread-local message of the last failed call ("" if none). */
const char* nr_last_error(void);

/* Residency checks.  Every entry point verifies that the pointers it hands to
 * a kernel are device (or managed) memory and fails with NR_ERR_INVALID naming
 * the argument otherwise.  Verified allocations are remembered per thread as
 * address ranges; nr_residency_flush() drops every thread's ranges (call it
 * after freeing device memory back to the driver, e.g. after
 * torch.cuda.empty_cache(), so a reused address is verified again).
 * nr_is_device_pointer(p) = 1 when p passes the same check, else 0. */
int nr_residency_flush(void);
int nr_is_device_pointer(const void* p);

/*
 * C[M, N] = epilogue(A[M, K] · W[N, K]ᵀ).
 * Replaces nn.Linear (+ F.relu / torch.exp / GEGLU / residual add) in
 *   FinalAttention.forward        modeling_utils.py:218-222
 *   LatentAttentionModel blocks   latent_attention.py:34-36, 59-61, 162-163
 * dtype_in NR_F32: exact-f32 MFMA (v_mfma_f32_32x32x2_f32);
 * dtype_in NR_BF16: bf16 MFMA (v_mfma_f32_32x32x16_bf16), f32 accumulate.
 * A and W share dtype_in; C is dtype_out; bias and R are f32 (bias nullable,
 * R only for NR_EPI_RESADD, R has dtype_out).  Requires N % 128 == 0,
 * K % 32 == 0 (f32) or K % 64 == 0 (bf16); M arbitrary.
 */
int nr_gemm(int dtype_in, int dtype_out, int epilogue, int64_t M, int64_t N, int64_t K,
            const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
            const void* R, int64_t ldr, void* C, int64_t ldc, void* stream);

/*
 * nr_gemm with the training-forward epilogue of FinalAttention
 * (modeling_utils.py:218-221: dropout(relu(linear(x))), p = 0.1 in train mode):
 *   C = relu(A·Wᵀ + bias) * keep(row, col) / (1 - p)
 * keep(idx = row * N + col) = field (idx & 3) of h >= round(p * 2^16), where h =
 * the splitmix64 finaliser of seed + (idx / 4 + 1) * 0x9E3779B97F4A7C15 and
 * field k = bits [16 k, 16 k + 16) (one hash per 4 consecutive elements;
 * restated in oracle/train_ref.py).  Replaces nn.Dropout's Philox stream: the
 * masks are a different (equally distributed; p quantised to 1/65536) draw,
 * reproducible from (seed, row, col).
 */
int nr_gemm_relu_dropout(int dtype_in, int dtype_out, int64_t M, int64_t N, int64_t K, const void* A,
                         int64_t lda, const void* W, int64_t ldw, const float* bias, void* C, int64_t ldc,
                         uint64_t seed, float p, void* stream);

/*
 * Data-grad GEMM through relu + dropout: C = Y > 0 ? (A·Wᵀ) * scale : 0, where
 * Y is the forward output relu(z) * keep / (1 - p) (so Y > 0 <=> z > 0 and kept)
 * and scale = 1 / (1 - p).  Y has dtype_out.
 */
int nr_gemm_drelu(int dtype_in, int dtype_out, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                  const void* W, int64_t ldw, const void* Y, int64_t ldy, void* C, int64_t ldc, float scale,
                  void* stream);

/*
 * Split-K fixup: C[r][c] = epi(sum_{s < parts} P[s][r][c] + bias[c]) over `rows` x N
 * (P: f32 [parts][rows][N], the K-slice partials of nr_gemm_grouped).  For the
 * last, partial round of 256x256 tiles of a GEMM (config-5 training at M % 4096
 * small): those rows run as `parts` K-slices side by side instead of one tile
 * per CU.  epilogue NR_EPI_NONE, NR_EPI_RELU_DROPOUT (mask of row row0 + r, p as
 * nr_gemm_relu_dropout, `scale` ignored), NR_EPI_DRELU (R = forward output,
 * C = R > 0 ? v * scale : 0), NR_EPI_RESADD (C = v + R) or NR_EPI_EXP
 * (C = exp(v)).  bias nullable.
 */
int nr_splitk_fixup(int dtype_out, int epilogue, int64_t rows, int64_t N, int parts, const float* partials,
                    const float* bias, const void* R, int64_t ldr, void* C, int64_t ldc, int64_t row0,
                    uint64_t seed, float p, float scale, void* stream);

/*
 * n independent C_i[M_i, N_i] = A_i · W_iᵀ (no bias, no epilogue) in ONE launch
 * over the union of the problems' 256x256 tiles (bf16 or exact-f32 in, f32 or bf16 out).
 * For problems too small to fill the 256 CUs alone: the config-5 weight-grad
 * GEMMs dW = dOutᵀ · X of FinalAttention's five linears (trainer.py:1044-1069
 * backward; four of them are 64 tiles each).  Arrays have n entries,
 * 1 <= n <= NR_GEMM_MAX_GROUP; each problem needs N % 256 == 0, K % 64 (bf16) / 32 (f32) == 0,
 * 16-B aligned operands and rows (as nr_gemm's 256x256 path).
 */
#define NR_GEMM_MAX_GROUP 8
int nr_gemm_grouped(int dtype_in, int dtype_out, int n, const int64_t* M, const int64_t* N, const int64_t* K,
                    const void* const* A, const int64_t* lda, const void* const* W, const int64_t* ldw,
                    void* const* C, const int64_t* ldc, void* stream);

/*
 * n independent C_i[M_i, N_i] = alpha_i A_i^T W_i in ONE launch, A_i [K_i][M_i]
 * and W_i [K_i][N_i] bf16 ROW-major (the reduction index is the row: lda / ldw
 * = row strides) -- the weight-grad GEMMs dW = dOut^T X of
 * AttentionAttentionTrainer's backward (trainer.py:1056-1057) on the row-major
 * activations, without transposed copies (LDS transposed reads).  C f32 or
 * bf16 (dtype_out).  M, N multiples of 256, K of 64; K = 0 leaves C untouched.
 * alpha nullable (all 1).
 */
int nr_gemm_grouped_tn(int dtype_out, int n, const int64_t* M, const int64_t* N, const int64_t* K,
                       const void* const* A, const int64_t* lda, const void* const* W, const int64_t* ldw,
                       void* const* C, const int64_t* ldc, const float* alpha, void* stream);

/*
 * y = LayerNorm(x) * gamma + beta over rows of `dim` (biased variance).
 * Replaces nn.LayerNorm in PreNorm latent_attention.py:10-12,16-19 and
 * MyLayer attention.py:165-166,193.  dim % 256 == 0, dim <= 2048.
 */
int nr_layernorm(int dtype_in, int dtype_out, int64_t rows, int64_t dim, const void* x,
                 int64_t ldx, const float* gamma, const float* beta, float eps, void* y,
                 int64_t ldy, void* stream);

/*
 * Gathered LayerNorm chain, f32 out:
 *   out[i] = LN_{n_ln-1}( ... LN_0(x[row_idx[i]]) ... ),  gammas/betas [n_ln][dim]
 * (nullable: gamma 1, beta 0), biased variance, f32 math.  row_idx nullable
 * (identity).  x may be NR_F32, NR_BF16 or NR_F16.
 * Replaces the token-attention encoder + last_token_pool of
 * FirstAttentionPoolFunc (modeling_utils.py:498-513 -> MyEncoder
 * attention.py:197-207, whose layers return g_mlp_layernorm(hidden_states),
 * attention.py:193, eps 1e-12 :155; last_token_pool modeling_utils.py:37-48):
 * with row_idx = the last valid token of each sequence only those rows are read.
 * dim in {256, 512, 1024, 2048}.
 */
int nr_gather_layernorm(int dtype_in, int64_t n, int64_t dim, const void* x, int64_t ldx,
                        const int64_t* row_idx, int n_ln, const float* gammas, const float* betas,
                        float eps, float* out, int64_t ldo, void* stream);

/*
 * In-place softmax over contiguous groups: x is f32 [rows][groups*64]
 * (row stride ldx), each run of 64 is one softmax.  Replaces the softmax
 * inside F.scaled_dot_product_attention at latent_attention.py:72
 * (64 latents per head).  dtype_out selects the element type of y.
 */
int nr_softmax64(int64_t rows, int64_t groups, const float* x, int64_t ldx, int dtype_out,
                 void* y, int64_t ldy, void* stream);

/*
 * out[r] = 1 / max(||x_r||_2, eps).  The per-row clamp of F.cosine_similarity
 * (data_model_helper.py:224-227, torch 2.10 semantics).
 */
int nr_row_inv_norm(int dtype, int64_t rows, int64_t dim, const void* x, int64_t ldx, float eps,
                    float* out, void* stream);

/*
 * Fused segmented history pooling + candidate cosine scoring.
 * Replaces get_final_attention_eval (data_model_helper.py:112-131: padded
 * batches through FinalAttention.forward modeling_utils.py:224-228 or
 * LatentAttentionModel.forward latent_attention.py:165-170) and the
 * per-impression F.cosine_similarity loop of get_cos_sim_scores
 * (data_model_helper.py:199-230).
 *
 * hist_table  per-news pooler table in `dtype`, row stride hist_ld:
 *             NR_POOL_FINAL : row = [x(dim) | exp(w)(dim)]
 *             NR_POOL_LATENT: row = h(dim)   (u = normalize(mean))
 *             NR_POOL_MEAN  : row = h(dim)   (u = mean)
 * cand_table  raw news embeddings [*, dim] in `dtype` (row stride cand_ld)
 * cand_inv_norm  f32 1/max(||cand_table row||, 1e-8)
 * hist_idx/hist_off, cand_idx/cand_off   CSR (int32 rows, int64 offsets,
 *             n_imp + 1 entries each).  hist_idx NULL: impression i pools the
 *             consecutive table rows hist_off[i] .. hist_off[i+1]-1.
 *             cand_off NULL: pooling only (no candidate is read; users required).
 * scores      f32 [cand_off[n_imp]] in impression order
 * users       nullable f32 [n_imp][dim]: the pooled user vectors
 *             (FinalAttention output / normalized latent mean / mean)
 * Supported dim: 1024 (NR_ERR_UNSUPPORTED otherwise; the reference's
 * EMBEDDING_DIM == 4096 latent branch, latent_attention.py:89-97, has no kernel).
 * Row indices are not bounds-checked: they must address rows of the tables.
 */
int nr_pool_score(int pooler, int dtype, int64_t dim, const void* hist_table, int64_t hist_ld,
                  const void* cand_table, int64_t cand_ld, const float* cand_inv_norm,
                  const int32_t* hist_idx, const int64_t* hist_off, const int32_t* cand_idx,
                  const int64_t* cand_off, int64_t n_imp, float* scores, float* users,
                  void* stream);

/*
 * Candidate scoring against stored user vectors: score_c = (u . e_c) /
 * max(|u|, 1e-8) * cand_inv_norm[c] with u = users[user_idx[i]] (f32 rows of
 * dim), for impressions that share a history (MIND: one history per user
 * across the user's impressions).  users is the `users` output of an
 * nr_pool_score pooling-only call (cand_off NULL) over the DISTINCT histories;
 * the scores are then bit-identical to nr_pool_score's fused pass, which
 * re-gathers a shared history once per impression.  Same tables, CSR and
 * dim rules as nr_pool_score.
 */
int nr_score_users(int dtype, int64_t dim, const float* users, const int32_t* user_idx, const void* cand_table,
                   int64_t cand_ld, const float* cand_inv_norm, const int32_t* cand_idx, const int64_t* cand_off,
                   int64_t n_imp, float* scores, void* stream);

/*
 * Dense descending rank per impression: ranks[c] = 1 + number of distinct
 * scores of the same impression that are strictly greater.  Bit-exact
 * restatement of scipy.stats.rankdata(-x, method="dense") used by
 * rank_group_preds (data_utils.py:414-415).  Impressions must have at most
 * 2048 candidates (MIND has <= 300): a larger one is not ranked and sets
 * *status = NR_ERR_UNSUPPORTED (`status`: a caller-zeroed int32 on the device,
 * checked by the Python wrapper, which raises).
 */
int nr_dense_rank(const float* scores, const int64_t* cand_off, int64_t n_imp, int32_t* ranks,
                  int32_t* status, void* stream);

/*
 * MIND metrics per impression from dense ranks (nr_dense_rank) and 0/1 labels
 * (replaces evaluation.score_row, evaluation.py:34-54, run per
 * impression by score(), :57-98).  metrics [n_imp][4] f64 = (AUC, MRR, nDCG@5,
 * nDCG@10); AUC = Mann-Whitney U / (P N) on 1 / rank (sklearn's ROC AUC, NaN for
 * single-class impressions).  MRR / nDCG are exact when the impression has no
 * tied ranks; tie_flag[i] = 1 marks impressions with ties (the reference's
 * positions then follow numpy's unstable argsort: evaluate those on the host).
 * status (caller-zeroed device int32): |1 if an impression has > 2048
 * candidates, |2 for a non-0/1 label or out-of-range rank (row set to NaN, flagged).
 */
int nr_impression_metrics(const int32_t* ranks, const float* labels, const int64_t* cand_off, int64_t n_imp,
                          double* metrics, int32_t* tie_flag, int32_t* status, void* stream);

/*
 * FinalAttention per-news transform for n news rows of `emb`:
 *   x = W3·relu(W2·relu(W1·e + b1) + b2) + b3 ;  p = exp(W5·relu(W4·x + b4))
 * written as table[n][2][1024] = (x, p) in `dtype` (modeling_utils.py:218-224,
 * computed once per unique news instead of per padded history slot).
 * Weights in `dtype` (torch layout), biases f32.  ws must hold
 * nr_final_attn_workspace_bytes(dtype, n) bytes.
 */
int64_t nr_final_attn_workspace_bytes(int dtype, int64_t n);
int nr_final_attn_transform(int dtype, int64_t n, const void* emb, int64_t emb_ld,
                            const void* W1, const float* b1, const void* W2, const float* b2,
                            const void* W3, const float* b3, const void* W4, const float* b4,
                            const void* W5, void* table, void* ws, int64_t ws_bytes,
                            void* stream);

/*
 * LatentAttentionModel per-news transform (latent_attention.py:157-163, K/V of
 * the 64 latents folded into the query and output projections once per model):
 *   y  = LN_q(e);  P = softmax_64(y · Aᵀ) per head;  h1 = e + P · Btᵀ
 *   h  = h1 + W2 · GEGLU(W1i · LN_f(h1) + b1i) + b2
 * A  [512][1024] rows h*64+j = (K_h[j] · W_q,h) / sqrt(512)   (K,V = to_kv(LN_c(latents)))
 * Bt [1024][512] column h*64+j = W_o,h · V_h[j]
 * W1i/b1i are W_1/b_1 with rows interleaved in 32-row (a, g) blocks.
 * Output table [n][1024] in `dtype`.  ws: nr_latent_workspace_bytes(dtype, n).
 */
int64_t nr_latent_workspace_bytes(int dtype, int64_t n);
int nr_latent_transform(int dtype, int64_t n, const void* emb, int64_t emb_ld,
                        const float* lnq_g, const float* lnq_b, const void* A, const void* Bt,
                        const float* lnf_g, const float* lnf_b, const void* W1i,
                        const float* b1i, const void* W2, const float* b2, void* table,
                        void* ws, int64_t ws_bytes, void* stream);

/*
 * The same transform for dtype == NR_BF16 with both LayerNorms folded into the
 * GEMM that consumes them (no normalised rows are written):
 *   LN(x) · Wᵀ = rstd ⊙ (x · W'ᵀ − mean ⊗ u) + c,
 *   W' = W ∘ γ (bf16),  u_n = Σ_k W'_nk (of the bf16 W'),  c_n = Σ_k β_k W_nk (+ bias)
 * with per-row (mean, rstd) from nr_row_stats.  Aq = A ∘ γ_q [512][1024],
 * ucq = (u[512], c[512]) f32; W1f = W1i ∘ γ_f [8192][1024] (interleaved rows),
 * ucf = (u[8192], c[8192]) f32 with c including b1i.  Bt, W2, b2 as above.
 * NR_ERR_UNSUPPORTED for NR_F32 (the f32 parity path keeps nr_latent_transform).
 */
int nr_latent_transform_lnfold(int dtype, int64_t n, const void* emb, int64_t emb_ld, const void* Aq,
                               const float* ucq, const void* Bt, const void* W1f, const float* ucf,
                               const void* W2, const float* b2, void* table, void* ws, int64_t ws_bytes,
                               void* stream);

/*
 * Per-row LayerNorm statistics out[r] = (mean, 1/sqrt(var + eps)) (f32 pairs,
 * biased variance: torch.nn.LayerNorm, latent_attention.py:11-13) of rows
 * [rows][1024] in `dtype`.
 */
int nr_row_stats(int dtype, int64_t rows, int64_t dim, const void* x, int64_t ldx, float eps, float* out,
                 void* stream);

/*
 * Title encoder pieces (XLM-R-large / e5-large-instruct), packed varlen tokens.
 * Replaces transformers XLMRobertaEmbeddings.forward (word + token_type +
 * position embeddings, LayerNorm) and the self-attention core
 * softmax(q kᵀ / sqrt(64)) v with the key-padding mask, as run by
 * get_text_embed_eval (modeling_utils.py:282-300).  The layer GEMMs use
 * nr_gemm (NR_EPI_RESADD / NR_EPI_GELU), the post-LNs nr_layernorm, and the
 * masked mean (+ F.normalize) (average_pool, modeling_utils.py:55-59,
 * data_model_helper.py:65-78) is nr_pool_score with NR_POOL_MEAN (NR_POOL_LATENT)
 * over consecutive token rows; nr_encoder_forward (below) chains all of it.
 *
 * nr_embed_ln: out[t] = LN(word[ids[t]] + type[0] + pos_emb[pos[t]]), dim 1024.
 * nr_attention_varlen: qkv [T][3072] (q | k | v, 16 heads x 64 per part),
 *   cu_seqlens int32 [n_seq+1], qblock_off int32 [n_seq+1] = prefix sum of
 *   ceil(L_i / 32), n_qblocks >= qblock_off[n_seq] (an upper bound is allowed:
 *   the exact count is read on the device), n_qblocks < 2^22; ctx [T][1024].
 */
int nr_embed_ln(int dtype, int64_t n_tokens, const int32_t* ids, const int32_t* pos, const void* word,
                const void* pos_emb, const void* type_emb, const float* gamma, const float* beta, float eps,
                void* out, void* stream);
int nr_attention_varlen(int dtype, int32_t n_seq, int64_t n_qblocks, const void* qkv,
                        const int32_t* cu_seqlens, const int32_t* qblock_off, void* ctx, void* stream);

/*
 * ---- Training step of config 5 (scripts/train_v3.py ->
 * AttentionAttentionTrainer.train_one_epoch, trainer.py:1030-1117) ----------
 * FinalAttention runs once per VALID history slot (the reference runs it per
 * padded slot and masks; padded slots carry zero gradient), slots packed in
 * CSR order (off[b]..off[b+1]) and padded with zero rows up to a multiple of
 * 64 so every weight-grad GEMM has K % 64 == 0.
 */

/* dst[i] = src[idx[i]] (idx NULL: identity; idx[i] < 0: zero row), dtype cast.
 * The history gather first_res[hist_indices] * mask (trainer.py:1052-1054). */
int nr_gather_rows(int dtype_in, int dtype_out, int64_t n, int64_t dim, const void* src, int64_t lds,
                   const int32_t* idx, void* dst, int64_t ldd, void* stream);

/* dst[c][r] = src[r][c] (dtype cast allowed): the operands of the data-grad
 * (dY·W = dY·(Wᵀ)ᵀ) and weight-grad (dYᵀ·X) GEMMs on the C = A·Wᵀ kernel. */
int nr_transpose(int dtype_in, int dtype_out, int64_t rows, int64_t cols, const void* src, int64_t lds,
                 void* dst, int64_t ldd, void* stream);

/* FinalAttention pooling forward over consecutive rows of xp = [x | exp(w)]
 * (row stride ld >= 2048, modeling_utils.py:224-228):
 * users[b] = sum x p / (sum p + 1e-10), z[b] = sum p + 1e-10 (both f32 [n_seg][1024]). */
int nr_final_pool_fwd(int dtype, int64_t n_seg, const int64_t* off, const void* xp, int64_t ld, float* users,
                      float* z, void* stream);

/* Its backward: dx_i = du p_i / z, dw_i = du (x_i - u) p_i / z (w = pre-exp
 * logit).  Rows off[n_seg]..n_rows-1 (padding) are zeroed. */
int nr_final_pool_bwd(int dtype, int64_t n_seg, const int64_t* off, int64_t n_rows, const void* xp, int64_t ld,
                      const float* users, const float* z, const float* du, void* dx, int64_t lddx, void* dw,
                      int64_t lddw, void* stream);

/* s_pos = cos(users[b], E[pos[b]]), s_neg = cos(users[b], E[neg[b]])
 * (F.cosine_similarity, per-vector clamp 1e-8, trainer.py:1058-1061) and
 * MarginRankingLoss(margin)(s_pos, s_neg, 1) = mean clamp_min(margin - s_pos + s_neg, 0)
 * (trainer.py:985,1063-1066).  *loss += the mean (caller zeroes it); du written;
 * dE rows accumulated (atomics, caller zeroes dE); s_out [2B] nullable. */
int nr_cosine_margin(int64_t B, const float* users, const float* E, int64_t lde, const int32_t* pos,
                     const int32_t* neg, float margin, float* s_out, float* loss, float* du, float* dE,
                     void* stream);

/* dst[idx[i]] += src[i] (f32 atomics; idx < 0 skipped): the gradient of the
 * history gather back to the unique-news rows. */
int nr_scatter_add_rows(int dtype, int64_t n, int64_t dim, const void* src, int64_t lds, const int32_t* idx,
                        float* dst, int64_t ldd, void* stream);

/* out[c] += sum_r src[r][c] (bias gradients; caller zeroes out). */
int nr_col_sum(int dtype, int64_t rows, int64_t cols, const void* src, int64_t lds, float* out, void* stream);

/* Token-model LayerNorm parameter grads (E = LN(x[row_idx]) g + b):
 * dgamma += sum dE xhat, dbeta += sum dE.  dim 1024; x f32 / bf16 / f16. */
int nr_ln_param_grad(int dtype_in, int64_t n, int64_t dim, const void* x, int64_t ldx, const int64_t* row_idx,
                     float eps, const float* dy, int64_t lddy, float* dgamma, float* dbeta, void* stream);

/* LatentAttentionModel training (f32; latent_attention.py:157-163 through autograd):
 * PreNorm LayerNorm input gradient (stats recomputed from x, dim 1024):
 * dx = rstd (dxh - mean(dxh) - xhat mean(dxh xhat)) [+ dres], dxh = dy gamma
 * (gamma NULL = 1; dres may alias dx). */
int nr_layernorm_bwd(int64_t n, int64_t dim, const float* x, int64_t ldx, const float* gamma, float eps,
                     const float* dy, int64_t lddy, const float* dres, int64_t ldr, float* dx, int64_t lddx,
                     void* stream);

/* Softmax backward over groups of 64 columns (one head's 64 latents):
 * ds = p (dp - sum_group(p dp)); ds f32 or bf16 (dtype_out). */
int nr_softmax64_bwd(int dtype_out, int64_t rows, int64_t cols, const float* p, int64_t ldp, const float* dp,
                     int64_t lddp, void* ds, int64_t ldds, void* stream);

/* GEGLU (latent_attention.py:24-27, exact-erf gelu): z = a gelu(g) with
 * a = G[:, :f], g = G[:, f:]; backward dG = [dz gelu(g), dz a gelu'(g)].  Inputs f32;
 * z / dG f32 or bf16 (dtype_out: the bf16-operand training mode's GEMM inputs). */
int nr_geglu_fwd(int dtype_out, int64_t rows, int64_t f, const float* g, int64_t ldg, void* z, int64_t ldz,
                 void* stream);
int nr_geglu_bwd(int dtype_out, int64_t rows, int64_t f, const float* g, int64_t ldg, const float* dz, int64_t lddz,
                 void* dg, int64_t lddg, void* stream);

/* *out += sum x^2 (the global grad norm of clip_grad_norm_, trainer.py:1067-1071). */
int nr_sumsq(int64_t n, const float* x, float* out, void* stream);

/* torch.optim.AdamW step (trainer.py:979-983: lr 1e-6, betas (0.9, 0.999),
 * eps 1e-8, weight_decay 0.01) over a flat f32 parameter buffer, with the
 * clip_grad_norm_(max_norm) coefficient min(max_norm / (sqrt(*sumsq) + 1e-6), 1)
 * folded in (sumsq NULL: no clipping).  p_bf16 (nullable) receives a bf16
 * copy of the updated parameters. */
int nr_adamw(int64_t n, float* p, const float* g, float* m, float* v, void* p_bf16, int64_t step, float lr,
             float beta1, float beta2, float eps, float weight_decay, float max_norm, const float* sumsq,
             void* stream);

/*
 * ---- Config-5 step with the latent pooler (BASELINE configs[4]: token encoder
 * + LatentAttentionModel, bf16 MFMA backward), forward + backward of one batch
 * as ONE call: the body of train_one_epoch (trainer.py:1044-1066) with
 * LatentAttentionModel (latent_attention.py:134-171) in FinalAttention's slot.
 *   E     = LN_tok(tok_last)                      (g_mlp_layernorm, eps 1e-12)
 *   fold  KV = LN_c(latents) Wkv^T; A_h = K_h Wq_h / sqrt(512); Bt_h^T = V_h Wo_h^T
 *   per history slot: X = LN_q(E[hist]); P = softmax64(X A^T); H1 = P Bt^T + E[hist]
 *                     G = LN_f(H1) W1^T + b1; Z = GEGLU(G)
 *   per batch row:    m = mean(Z) W2^T + b2 + mean(H1)   (= mean(H): the last
 *                     linear layer commutes with the history mean)
 *                     u = normalize(m); loss = MarginRankingLoss(2)(cos(u, E[pos]), cos(u, E[neg]))
 * and the exact backward of all of it; every gradient is written into its f32
 * grad buffer (the step zeroes the ones it accumulates itself).  The weight
 * grads of W1 / W2 run on an internal second stream beside the data-grad
 * chain, joined back to `stream` (event wait) before the call returns, so the
 * step stays ordered on `stream` and graph-capturable.  dtype
 * NR_F32: exact-f32 MFMA GEMMs and f32 activations; NR_BF16: bf16 operands and
 * activations, f32 accumulation, statistics and parameter gradients.
 * Weights are passed in `dtype` (the bf16 mirror for NR_BF16), LayerNorm
 * parameters, biases and latents in f32.  hist_idx: [Hs] indices into the U
 * rows, hist_off [B+1] CSR offsets, pos / neg [B].  users (nullable, f32
 * [B][1024]): the normalized pooled users.  ws: nr_latent_train_workspace_bytes.
 * CSR contract (not checked on the device): hist_off[0] = 0, hist_off[B] = Hs,
 * non-decreasing, every row non-empty; 0 <= hist_idx[i] < U.  Both the per-slot
 * kernels (Hs valid rows) and the per-row means (hist_off) rely on it.
 */
typedef struct nr_latent_train_args {
  int dtype;
  int tok_dtype;  /* NR_F32 / NR_BF16 / NR_F16 */
  int64_t B, U, Hs;
  const void* tok_last; /* [U][1024] last valid token state per unique news */
  const int32_t* hist_idx;
  const int64_t* hist_off;
  const int32_t* pos;
  const int32_t* neg;
  float margin;
  /* parameters (f32 unless noted) */
  const float *tok_g, *tok_b; /* token LayerNorm (g_mlp_layernorm) */
  const float* latents;       /* [64][1024] */
  const float *nq_g, *nq_b;   /* cross_attend_blocks.0.norm */
  const float *nc_g, *nc_b;   /* cross_attend_blocks.0.norm_context */
  const void *Wq, *Wkv, *Wo;  /* `dtype`: to_q [4096][1024], to_kv [8192][1024], to_out [1024][4096] */
  const float *nf_g, *nf_b;   /* cross_attend_blocks.1.norm */
  const void* W1;             /* `dtype`: net.0.weight [8192][1024] */
  const float* b1;            /* [8192] */
  const void* W2;             /* `dtype`: net.2.weight [1024][4096] */
  const float* b2;            /* [1024] */
  /* gradients (f32, same shapes; fully written by the step) */
  float *g_tok_g, *g_tok_b, *g_latents, *g_nq_g, *g_nq_b, *g_nc_g, *g_nc_b, *g_Wq, *g_Wkv, *g_Wo;
  float *g_nf_g, *g_nf_b, *g_W1, *g_b1, *g_W2, *g_b2;
  /* outputs */
  float* loss;  /* device scalar (set, not accumulated) */
  float* users; /* nullable [B][1024] */
  float* sumsq; /* nullable device scalar: set to the squared L2 norm of all the
                   gradients above (the clip's input to nr_adamw) */
} nr_latent_train_args;

int64_t nr_latent_train_workspace_bytes(int dtype, int64_t B, int64_t U, int64_t Hs);
int nr_latent_train_step(const nr_latent_train_args* args, void* ws, int64_t ws_bytes, void* stream);

/*
 * ---- Config-5 step with FinalAttention (the pairing scripts/train_v3.py runs:
 * AttentionAttentionTrainer.train_one_epoch, trainer.py:1044-1066, with
 * FinalAttention.forward, modeling_utils.py:195-228, in train mode), forward +
 * backward of one batch as ONE call:
 *   E  = LN_tok(tok_last)                              (g_mlp_layernorm, eps 1e-12)
 *   per history slot: S = E[hist]; X1 = drop(relu(S W1^T + b1)); X2 = drop(relu(X1 W2^T + b2))
 *                     X = X2 W3^T + b3; Y = drop(relu(X W4^T + b4)); P = exp(Y W5^T)
 *   per batch row:    u = sum X P / (sum P + 1e-10)  (per dimension)
 *                     loss = MarginRankingLoss(margin)(cos(u, E[pos]), cos(u, E[neg]))
 * and the exact backward; every gradient is written into its f32 grad buffer.
 * Dropout p on the three ReLU layers from the counter-hash stream of
 * nr_gemm_relu_dropout with seed[0..2] (p = 0: the reference's eval-identical
 * step).  The weight transposes run on an internal side stream joined back to
 * `stream`, so the step stays ordered on `stream`.  dtype NR_F32: exact-f32 MFMA
 * and f32 activations (the parity mode); NR_BF16: bf16 operands / activations,
 * f32 accumulation, statistics and gradients, the bias grads summed from the
 * f32 GEMM results before rounding, the weight grads read from the row-major
 * activations (nr_gemm_grouped_tn's kernel).  Weights W1..W5 in `dtype` (the
 * bf16 mirror for NR_BF16), biases and the token LN parameters f32.  CSR
 * contract as nr_latent_train_step (hist_off[0] = 0, hist_off[B] = Hs,
 * non-empty rows, 0 <= hist_idx < U).  users (nullable, f32 [B][1024]): the
 * pooled users.  ws: nr_final_train_workspace_bytes, 256-byte aligned.
 */
typedef struct nr_final_train_args {
  int dtype;
  int tok_dtype; /* NR_F32 / NR_BF16 / NR_F16 */
  int64_t B, U, Hs;
  const void* tok_last; /* [U][1024] */
  const int32_t* hist_idx;
  const int64_t* hist_off;
  const int32_t* pos;
  const int32_t* neg;
  float margin;
  float p;           /* dropout probability of the three ReLU layers */
  uint64_t seed[3];  /* their dropout streams */
  const float *tok_g, *tok_b;
  const void* W1; const float* b1; /* linear1 [4096][1024] */
  const void* W2; const float* b2; /* linear2 [4096][4096] */
  const void* W3; const float* b3; /* linear3 [1024][4096] */
  const void* W4; const float* b4; /* linear4 [4096][1024] */
  const void* W5;                  /* linear5 [1024][4096], no bias */
  float *g_tok_g, *g_tok_b, *g_W1, *g_b1, *g_W2, *g_b2, *g_W3, *g_b3, *g_W4, *g_b4, *g_W5;
  float* loss;  /* device scalar (set, not accumulated) */
  float* users; /* nullable [B][1024] */
  float* sumsq; /* nullable device scalar: set to the sum of squares of every gradient written (the
                   clip_grad_norm_ input; nr_adamw's `sumsq`), summed on the fly in bf16 mode */
} nr_final_train_args;

int64_t nr_final_train_workspace_bytes(int dtype, int64_t B, int64_t U, int64_t Hs);
int nr_final_train_step(const nr_final_train_args* args, void* ws, int64_t ws_bytes, void* stream);

/*
 * ---- RCCL communicator of the multi-GPU eval (SURVEY §8(b) nr_allgather,
 * §8(e)): one process per GPU; every rank transforms a row shard of the
 * per-news table and ONE all-gather over xGMI gives each GPU the whole table.
 * The reference has no distributed code: this is the exchange
 * step the north star adds.  RCCL is resolved at run time (the process's
 * librccl.so.1, e.g. the one torch mapped); without it the entries return
 * NR_ERR_UNSUPPORTED.
 *   rank 0: nr_comm_unique_id(id); the host sends the 128 id bytes to every
 *   rank (any channel: torch.distributed broadcast, a file, MPI ...);
 *   every rank: nr_init(device); nr_comm_init(&c, id, nranks, rank)
 *   (collective: blocks until all nranks have called it).
 * nr_comm_init_timeout: the same with a deadline.  timeout_ms > 0 forms a
 *   non-blocking RCCL communicator (ncclCommInitRankConfig, blocking = 0) and
 *   polls it; if it has not formed within timeout_ms (a peer never joined or
 *   died inside its init) it is aborted (ncclCommAbort) and the call returns
 *   NR_ERR_TIMEOUT, so a stuck rank fails with a record instead of hanging.
 *   timeout_ms <= 0, or an RCCL without the non-blocking entries: as nr_comm_init.
 * nr_allgather: recv[r * bytes_per_rank ..] = rank r's send, async on `stream`;
 * in place when send == recv + rank * bytes_per_rank.
 */
#define NR_COMM_ID_BYTES 128
typedef struct nr_comm* nr_comm_t;
int nr_rccl_version(void); /* RCCL's NCCL_VERSION_CODE, 0 when RCCL is absent */
int nr_comm_unique_id(unsigned char* id);
int nr_comm_init(nr_comm_t* comm, const unsigned char* id, int nranks, int rank);
int nr_comm_init_timeout(nr_comm_t* comm, const unsigned char* id, int nranks, int rank, int64_t timeout_ms);
int nr_comm_destroy(nr_comm_t comm);
int nr_allgather(nr_comm_t comm, const void* send, void* recv, int64_t bytes_per_rank, void* stream);

/*
 * ---- Whole title-encoder forward (get_embeddings, data_model_helper.py:45-84:
 * get_embed_from_model -> get_text_embed_eval modeling_utils.py:282-323 ->
 * XLMRobertaModel -> average_pool (+ F.normalize for e5-instruct)) ----------
 * Packed varlen tokens, no padding: sequence i is ids[cu_i .. cu_i + seq_lens[i]),
 * cu = prefix sum of seq_lens (computed on the device).  Positions follow
 * transformers' create_position_ids_from_input_ids (pad id 1: pad + cumsum(id
 * != pad) * (id != pad)).  Per layer (post-LN BERT, eps `eps`):
 *   x = LN1(Attn(x Wqkvᵀ + bqkv) Woᵀ + bo + x);  x = LN2(gelu(x W1ᵀ + b1) W2ᵀ + b2 + x)
 * `layers` is a HOST array of n_layers descriptors of device weights (torch
 * nn.Linear layout, `dtype`; biases and LN parameters f32).  Output:
 *   pool NR_POOL_MEAN   pooled [n_seq][1024] f32 = average_pool(last_hidden_state)
 *   pool NR_POOL_LATENT pooled = F.normalize(average_pool(...), p=2, eps=1e-12)
 *   pool NR_POOL_NONE   no pooled output
 * hidden (nullable, [n_tokens][1024] `dtype`): the packed last_hidden_state.
 * ids and seq_lens are device int32 arrays (seq_lens[i] >= 1); n_tokens = their
 * sum.  status (nullable, caller-zeroed device int32): |1 a position id
 * reached n_positions (clamped), |2 a token id outside [0, vocab) (clamped).
 * ws: nr_encoder_workspace_bytes(dtype, n_tokens, n_seq) bytes.
 */
typedef struct nr_encoder_layer {
  const void* wqkv;    /* [3072][1024]: self.query | self.key | self.value weights */
  const float* bqkv;   /* [3072] */
  const void* wo;      /* attention.output.dense [1024][1024] */
  const float* bo;
  const float* ln1_g;  /* attention.output.LayerNorm */
  const float* ln1_b;
  const void* w1;      /* intermediate.dense [4096][1024] */
  const float* b1;
  const void* w2;      /* output.dense [1024][4096] */
  const float* b2;
  const float* ln2_g;  /* output.LayerNorm */
  const float* ln2_b;
} nr_encoder_layer;

int64_t nr_encoder_workspace_bytes(int dtype, int64_t n_tokens, int64_t n_seq);
int nr_encoder_forward(int dtype, int n_layers, const nr_encoder_layer* layers, const void* word_emb,
                       int64_t vocab, const void* pos_emb, int64_t n_positions, const void* type_emb,
                       const float* emb_ln_g, const float* emb_ln_b, float eps, int64_t n_seq,
                       int64_t n_tokens, const int32_t* seq_lens, const int32_t* ids, int pool, float* pooled,
                       void* hidden, int32_t* status, void* ws, int64_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NEWSREC_H */
