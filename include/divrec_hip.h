/*
 * libdivrec_hip — C ABI of the MI355X (gfx950) hot path of divrec
 * (amtsyplov/diversity-recommendations). Plain pointers and sizes only; no
 * torch types. Every pointer argument is DEVICE memory owned by the caller
 * unless the comment says otherwise. The library never allocates device
 * memory: scratch comes from a caller-owned workspace sized by the matching
 * *_workspace() query. All work is enqueued asynchronously on `stream`
 * (a hipStream_t; NULL = the legacy default stream).
 *
 * Return value: DR_OK (0) or a negative DR_E* code; dr_last_error() then holds
 * a thread-local message. The Python host (divrec/_backend.py) raises
 * RuntimeError(dr_last_error()) on any non-zero status.
 *
 * Reference entry points each function replaces are cited as
 * path:line relative to the reference tree (divrec/ ...).
 */
#ifndef DIVREC_HIP_H_
#define DIVREC_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* dr_stream_t; /* hipStream_t */

enum dr_status {
  DR_OK = 0,
  DR_EINVAL = -1,       /* bad shape / pointer / argument */
  DR_EUNSUPPORTED = -2, /* unsupported d / k / dtype combination */
  DR_EHIP = -3,         /* HIP runtime error (launch failure etc.) */
  DR_EWORKSPACE = -4    /* workspace too small */
};

enum dr_dtype { DR_F32 = 0, DR_BF16 = 1, DR_I32 = 2, DR_I64 = 3, DR_F64 = 4 };

enum dr_ild_kind {
  DR_ILD_COSINE = 0,    /* 1 - <e_i,e_j> / (|e_i| |e_j|) */
  DR_ILD_DOT = 1,       /* <e_i,e_j> */
  DR_ILD_EUCLIDEAN = 2  /* |e_i - e_j|_2 */
};

/* Library version (major*10000 + minor*100 + patch). */
int dr_version(void);
/* Build id: the first 16 hex digits of a sha256 over the library's source files
 * (the .hip and .h files of csrc/ and include/), baked in at compile time, so a run can
 * show which sources the loaded library was built from. */
const char* dr_build_id(void);
/* Thread-local message of the last failing call on this thread ("" if none). */
const char* dr_last_error(void);

/* Planner knobs: process-wide overrides of dr_score_topk's launch planner (and
 * of dr_mmr_rerank's grid, DR_KNOB_SCAN_SLOTS), for tests and A/B timing runs
 * only. Every plan gives identical results; only the time differs. The
 * library reads no environment variable: a knob holds the default plan until
 * it is set here, and value NaN restores the default. Thread-safe (atomic). */
enum dr_plan_knob {
  DR_KNOB_SCAN_SLOTS = 0,   /* workgroup slots planned for (split-tail plans at small sizes) */
  DR_KNOB_SCAN_SPLIT = 1,   /* max catalog chunks of a tail block (1 = no split) */
  DR_KNOB_TAIL_KEYS = 2,    /* finalize key cap of a split-tail user */
  DR_KNOB_SCAN_SEED = 3,    /* 0: never seed from a sample; 1: always (>= 2^18 rows) */
  DR_KNOB_GUESS_STRIDE = 4, /* sample stride of the guessed thresholds */
  DR_KNOB_GUESS_Z1 = 5,     /* set: ks1 = mu + z sigma + c1 instead of the 0.5 % Poisson-tail rank */
  DR_KNOB_GUESS_C1 = 6,     /* set: the offset c1 of that form (z defaults to 3) */
  DR_KNOB_GUESS_TIGHT = 7,  /* 0: one tier (ks1 = ks) */
  DR_KNOB_SAMPLE_DENSE = 8, /* 0: sample scan on compacted key buffers, not dense tile maxima; >1: budget GiB */
  DR_KNOB_ILD_STREAM = 9,   /* dr_ild_embedding, k <= 128: 0 = one wave per user, 1 = streamed persistent grid (default: streamed for d = 128 cosine / dot, k > 40) */
  DR_KNOB_ILD_BUFS = 10,    /* streamed ILD: ring slots (1-KB row pieces) per wave, at least one list's (default: as many as LDS allows) */
  DR_KNOB_COUNT = 11
};
/* Set knob `knob` to `value` (NaN = default). DR_EINVAL for an unknown knob,
 * an infinite value or one outside the knob's range: SCAN_SLOTS, SCAN_SPLIT,
 * TAIL_KEYS and GUESS_STRIDE take integers in [1, 2^30]; SCAN_SEED, GUESS_TIGHT
 * and ILD_STREAM 0 or 1; GUESS_Z1 / GUESS_C1 any finite value in [-64, 64];
 * SAMPLE_DENSE 0 (off), 1 (on, the default budget) or a budget in GiB above
 * 1 (up to 2^20); ILD_BUFS an
 * integer in [1, 64]. */
int dr_set_plan_knob(int knob, double value);
/* Current value of a knob (NaN = default; NaN for an unknown knob). */
double dr_get_plan_knob(int knob);

/* ---------------------------------------------------------------------------
 * Id range checks (all gather-type calls below): an id outside [0, rows) of
 * its table — what nn.Embedding / tensor indexing reject with IndexError in
 * the reference — is never dereferenced. The affected unit (pair, triple,
 * user) produces NaN / adds nothing, and *err (caller-zeroed int32, may be
 * NULL) is incremented once per such unit. The host raises IndexError when
 * it reads a non-zero count.
 *
 * MatrixFactorization.forward: s[n] = sum_d U[user_id[n], d] * I[item_id[n], d]
 * Replaces divrec/models/matrix_factorization.py:26-28 (two nn.Embedding
 * lookups + torch.sum(u * i, dim=1)). Tables row-major [rows, d], dtype
 * DR_F32 or DR_BF16 (both tables the same dtype); ids int64; out fp32 [n].
 * Runs of equal ids (RankingDataset's full((n,), u), PairWiseDataset's m x m
 * pairs, divrec/datasets/base_datasets.py:94-107,165-171) read each row once.
 */
int dr_gather_dot(const void* user_table, int64_t n_user_rows, const void* item_table,
                  int64_t n_item_rows, int dtype, int64_t d, const int64_t* user_id,
                  const int64_t* item_id, int64_t n, float* out, int32_t* err,
                  dr_stream_t stream);

/* Backward of dr_gather_dot into DENSE fp32 gradient tables (nn.Embedding with
 * sparse=False, divrec/models/matrix_factorization.py:16-17):
 *   grad_user[user_id[n]] += grad_out[n] * I[item_id[n]]
 *   grad_item[item_id[n]] += grad_out[n] * U[user_id[n]]
 * Accumulates with fp32 atomics (order-dependent in the last bits). Either
 * grad pointer may be NULL to skip that table. Tables must be DR_F32. */
int dr_gather_dot_backward(const float* user_table, int64_t n_user_rows, const float* item_table,
                           int64_t n_item_rows, int64_t d, const int64_t* user_id,
                           const int64_t* item_id, int64_t n, const float* grad_out,
                           float* grad_user, float* grad_item, int32_t* err, dr_stream_t stream);

/* ---------------------------------------------------------------------------
 * Full-catalog scoring + top-K: for each of the n_users user rows, the k best
 * items of the catalog slice [item_base, item_base + n_items) by
 * score = <U[user], I[item]>. Replaces get_model_recommendations
 * (divrec/train/utils.py:53-77) over RankingDataset candidates
 * (divrec/datasets/base_datasets.py:136-171), which scores each candidate with
 * MatrixFactorization.forward (divrec/models/matrix_factorization.py:26-28).
 *
 * Ranking order is score descending, item id ascending (the deterministic
 * tie-break the reference's unstable argsort leaves undefined, utils.py:73).
 *
 *   dtype       DR_BF16: bf16 tables, bf16 MFMA (exact products, fp32 sums) —
 *               the fast mode; d in {32, 64, 128, 256, 512}.
 *               DR_F32: fp32 tables, fp32 MFMA (an exact fp32 fmaf chain per
 *               score, the reference's own arithmetic up to summation order) —
 *               the faithful mode; d in {32, 64, 128, 256}.
 *               Other widths: pad both tables with zero columns (exact).
 *   user_table  [*, d]; user_ids int64 [n_users] or NULL (rows 0..n_users-1)
 *   item_table  [n_items, d] (the rows of THIS slice; global id = item_base + row)
 *   1 <= k <= 1024
 *   excl_rowptr int64 [n_users + 1], excl_items int32 (GLOBAL item ids, sorted
 *     ascending per row): items excluded per user (RankingDataset `frozen`,
 *     base_datasets.py:143-149). Both NULL = no exclusion.
 *   out_scores fp32 [n_users, k], out_items int32 [n_users, k] (GLOBAL ids);
 *     slots with no candidate hold item -1 and score -inf.
 *   workspace of dr_score_topk_workspace(...) bytes (query with identical args,
 *     with the device that runs the call current: the launch plan, and with it
 *     the size, depends on the device's CU count). Its size: candidate buffers
 *     of n_users (rounded up to a user block) x CAP x 8 B (CAP 512, 1024 or
 *     2048 by d and k), plus rows for the extra chunks of a split tail; for
 *     catalogs of 2^18 rows or more (the guessed thresholds) that region is
 *     instead the sample scan's dense [users x sample tiles] fp32 tile-max
 *     matrix when that is larger and within the SAMPLE_DENSE budget (16 GiB by
 *     default; 1M x 10M at d = 128: 9.8 GB against 8.5 GB of buffers), plus
 *     about 40 B per user of thresholds and fail lists and a copy of the
 *     sample rows.
 */
size_t dr_score_topk_workspace(int64_t n_users, int64_t n_items, int dtype, int d, int k);
int dr_score_topk(const void* user_table, const int64_t* user_ids, int64_t n_users,
                  const void* item_table, int64_t n_items, int64_t item_base, int dtype, int d,
                  int k, const int64_t* excl_rowptr, const int32_t* excl_items,
                  float* out_scores, int32_t* out_items, void* workspace,
                  size_t workspace_bytes, dr_stream_t stream);

/* The launch plan dr_score_topk uses for these arguments on the current device
 * (host-only query, no device work; the planner knobs of dr_set_plan_knob
 * included), so tests can show which plan they exercised. out[0..11] = users per
 * workgroup, user blocks, head blocks (scanned whole), catalog chunks per tail
 * block (1 = no split), tail chunk length, grid, candidate capacity, sample
 * stride of the guessed threshold (0 = plain scan), sample rows, sample rank ks,
 * finalize keys of a head user, finalize keys of a tail user; with n_out >= 13,
 * out[12] = the first-tier rank ks1 <= ks the main scan starts from. n_out >= 12. */
int dr_score_topk_plan(int64_t n_users, int64_t n_items, int dtype, int d, int k, int64_t* out,
                       int n_out);

/* Guess statistics of the last dr_score_topk call on `workspace` with these
 * arguments (host query; synchronises with a copy): out[0] = users whose
 * first-tier guessed threshold failed (rescanned from their safe threshold),
 * out[1] = users every guess failed (rescanned from -inf). 0, 0 for plain
 * scans (catalogs below 2^18 rows). int32 out[2] is HOST memory. */
int dr_score_topk_fail_counts(const void* workspace, int64_t n_users, int64_t n_items, int dtype,
                              int d, int k, int32_t* out);

/* The guessed thresholds of the item-sharded multi-GPU top-k, computed like
 * dr_score_topk's own guess: sample_rows [n_sample, d] (dtype as the user
 * table) are the whole catalog's rows at the guess stride, gathered from every
 * shard; the whole 32-row tiles of them (n_sample rounded down) are scanned by
 * the tile-max sample scan, and thr1[u] / thr2[u] (fp32 [n_users], device)
 * are set strictly below the ks1-th / ks-th best tile-max score of user u
 * (-inf when there are fewer): lower bounds of the user's ks1-th / ks-th best
 * sample score, the first-tier and safe thresholds of
 * divrec.distributed.thresholded_exchange (replaces nothing in the reference:
 * the scale-out of divrec/train/utils.py:53-77). 1 <= ks1 <= ks <= 256.
 * Workspace of dr_sample_thresholds_workspace(...) bytes. */
size_t dr_sample_thresholds_workspace(int64_t n_users, int64_t n_sample, int dtype, int d, int ks);
int dr_sample_thresholds(const void* user_table, const int64_t* user_ids, int64_t n_users,
                         const void* sample_rows, int64_t n_sample, int dtype, int d, int ks1,
                         int ks, float* thr1, float* thr2, void* workspace, size_t workspace_bytes,
                         dr_stream_t stream);

/* dr_score_topk with caller-given per-user thresholds: the top-k (same order)
 * of the items whose score is STRICTLY above init_thr[u]; slots past the last
 * such item hold item -1 and score -inf. init_thr fp32 [n_users] (-inf = plain
 * top-k). The item-sharded multi-GPU top-k passes thresholds guessed from a
 * sample of the whole catalog, so each shard returns only items that can
 * reach the global top-k (divrec.distributed.sharded_score_topk; replaces the
 * per-shard share of divrec/train/utils.py:53-77). Other arguments as
 * dr_score_topk; workspace of dr_score_topk_seeded_workspace(...) bytes.
 */
size_t dr_score_topk_seeded_workspace(int64_t n_users, int64_t n_items, int dtype, int d, int k);
int dr_score_topk_seeded(const void* user_table, const int64_t* user_ids, int64_t n_users,
                         const void* item_table, int64_t n_items, int64_t item_base, int dtype,
                         int d, int k, const float* init_thr, const int64_t* excl_rowptr,
                         const int32_t* excl_items, float* out_scores, int32_t* out_items,
                         void* workspace, size_t workspace_bytes, dr_stream_t stream);

/* Merge `parts` per-user top-k lists (each sorted by the order above) into one:
 *   in_scores/in_items [parts, n_users, k_in] -> out [n_users, k_out], k_out <= parts*k_in
 *   (k_out <= 1024 when parts*k_in > 2048; entries with item -1 are empty).
 * This is the exchange step of the item-row-sharded top-K:
 * shard partials are exchanged over RCCL and merged here; the result is
 * bit-identical to the single-device dr_score_topk over the whole catalog. */
int dr_topk_merge(const float* in_scores, const int32_t* in_items, int parts, int64_t n_users,
                  int k_in, int k_out, float* out_scores, int32_t* out_items,
                  dr_stream_t stream);

/* ---------------------------------------------------------------------------
 * Intra-list diversity, IntraListDiversityScore.recommendations_loss with
 * reduction 'none' (divrec/losses/intra_list_diversity_score.py:20-42):
 *   out[u] = (sum_{p<q} D[r[u,p], r[u,q]]) / (k * (k - 1))     (k = 1 -> NaN)
 * `recs` [n_users, k] item ids of dtype rec_dtype (DR_I32 or DR_I64); a list
 * holding an id outside [0, n_items) gives NaN and counts in *err (above).
 */

/* Dense distance matrix D [n_items, n_items] (dtype DR_F32, DR_F64, DR_I32 or
 * DR_I64). Float D is accumulated in its own precision in itertools.combinations order, like the
 * reference's Python sum (bit-exact); integer D is summed exactly. */
int dr_ild_dense(const void* recs, int rec_dtype, int64_t n_users, int k, const void* dist,
                 int dist_dtype, int64_t n_items, float* out, int32_t* err, dr_stream_t stream);

/* The un-normalised pair sum of the same lists, sum_{p<q} D[r[u,p], r[u,q]], the
 * reference's IntraListDiversityScore.user_ild (:36-42): accumulated in D's
 * own precision in combinations order (fp32 D: the Python sum of 0-d fp32
 * tensors, bit-exact; integer D: exact), stored as double (k = 1: 0). */
int dr_ild_dense_pair_sum(const void* recs, int rec_dtype, int64_t n_users, int k,
                          const void* dist, int dist_dtype, int64_t n_items, double* out,
                          int32_t* err, dr_stream_t stream);

/* Label equality D[i,j] = (label[i] == label[j]), the matrix of
 * IntraListBinaryUnfairnessScore.get_distance_matrix (:60-63), computed on the
 * fly from labels int64 [n_items] (exact integer count). Any k: lists of up to
 * 1024 stage their labels in LDS, longer ones read them through the cache. */
int dr_ild_labels(const void* recs, int rec_dtype, int64_t n_users, int k,
                  const int64_t* labels, int64_t n_items, float* out, int32_t* err,
                  dr_stream_t stream);

/* Distance computed on the fly from an item embedding table (bf16 [n_items, d],
 * d in {32, 64, 128, 256}, 1 <= k <= 16384) by bf16 MFMA Gram tiles per user
 * (kind: enum dr_ild_kind). k <= 128: the list in registers, fp32 accumulation;
 * longer lists (the reference's user_ild takes any length): the row tiles
 * streamed through the cache, tile sums accumulated in double. */
int dr_ild_embedding(const void* recs, int rec_dtype, int64_t n_users, int k,
                     const void* item_table, int64_t n_items, int d, int kind, float* out,
                     int32_t* err, dr_stream_t stream);

/* ---------------------------------------------------------------------------
 * BPR step (pair_wise_train_loop, divrec/train/utils.py:144-152, with
 * LogSigmoidDifferenceLoss, divrec/losses/log_sigmoid_difference_loss.py:11-14):
 *   x[b] = <U[u_b], I[p_b]> - <U[u_b], I[n_b]>
 *   loss[b] = -logsigmoid(x[b]);  hit[b] = (x_pos >= x_neg) (AUCScore, auc_score.py:6-10)
 *   g = -sigmoid(-x) * grad_scale  (grad_scale = 1/B for the 'mean' reduction)
 *   grad_user[u] += g (I[p] - I[n]); grad_item[p] += g U[u]; grad_item[n] -= g U[u]
 * fp32 tables [*, d]; ids int64 [B]; loss fp32 [B] and hit int32 [B] may be
 * NULL. Gradients are DENSE fp32 tables accumulated with atomics. A triple
 * with an out-of-range id adds nothing, gets loss NaN / hit 0 and counts in
 * *err (id range checks, above). */
int dr_bpr_fwd_bwd(const float* user_table, int64_t n_user_rows, const float* item_table,
                   int64_t n_item_rows, int64_t d, const int64_t* user_id,
                   const int64_t* pos_id, const int64_t* neg_id, int64_t batch,
                   float grad_scale, float* loss, int32_t* hit, float* grad_user,
                   float* grad_item, int32_t* err, dr_stream_t stream);

/* Dense Adam step in fp32 over n elements, the update torch.optim.Adam
 * (amsgrad=False, maximize=False) applies at divrec/train/utils.py:151:
 *   g = grad + weight_decay * param; m = lerp(m, g, 1 - beta1);
 *   v = beta2 * v + (1 - beta2) * g * g;
 *   param -= (lr / (1 - beta1^step)) * m / (sqrt(v) / sqrt(1 - beta2^step) + eps)
 * `step` is the 1-based step count AFTER incrementing. Hyper-parameters are
 * doubles (Python floats); they are combined in double and cast to fp32 once,
 * as torch does. */
int dr_adam_dense(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                  int64_t n, double lr, double beta1, double beta2, double eps,
                  double weight_decay, int64_t step, dr_stream_t stream);

/* Row-sparse ("lazy") Adam, SURVEY.md §8f rank 3: the update
 * torch.optim.SparseAdam applies (torch/optim/_functional.py, sparse_adam) to
 * a coalesced sparse gradient with indices `rows` (unique, int64, [n_rows]) and
 * values grad[rows] read from a DENSE fp32 gradient table [*, d] (as
 * accumulated by dr_bpr_fwd_bwd). Only the listed rows of param / exp_avg /
 * exp_avg_sq change. zero_grad != 0 also zeroes grad[rows], leaving the table
 * all-zero for the next batch without a full memset. The reference trains with
 * dense Adam (divrec/train/utils.py:151 over sparse=False embeddings,
 * divrec/models/matrix_factorization.py:16-17); this is the opt-in alternative.
 * `step` is SparseAdam's state step AFTER incrementing. */
int dr_adam_rows(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t d,
                 const int64_t* rows, int64_t n_rows, double lr, double beta1, double beta2,
                 double eps, int64_t step, int zero_grad, dr_stream_t stream);

/* Device-side pairwise sampling, SURVEY.md §8f rank 4: the sampling of
 * PairWiseDataset.__iter__ (divrec/datasets/base_datasets.py:70-107) for the
 * users `users` [n_users] (int64 row ids), in that order:
 *   pos_out[b, :] = m draws with replacement, uniform over the user's unique
 *                   positives (CSR pos_rowptr [*+1] / pos_items int32, sorted);
 *   neg_out[b, :] = m draws with replacement, uniform over
 *                   [0, n_items) - positives - frozen (CSR excl_*, may be NULL),
 *                   by rejection (at most 4096 tries per draw);
 *   uid/pid/nid [n_users*m*m] int64 (optional, all or none): the m x m
 *                   Cartesian product, positive-major, as the reference yields it.
 * Draws come from a counter-based hash of (seed, user id, draw, try) instead of
 * Python's random stream: parity is distributional. *err_count (caller-zeroed)
 * counts failed draws: users without positives (the reference raises
 * IndexError) and negatives with an empty allowed set; their ids are -1. */
int dr_sample_pairwise(const int64_t* users, int64_t n_users, const int64_t* pos_rowptr,
                       const int32_t* pos_items, const int64_t* excl_rowptr,
                       const int32_t* excl_items, int64_t n_items, int m, uint64_t seed,
                       int32_t* pos_out, int32_t* neg_out, int64_t* uid, int64_t* pid,
                       int64_t* nid, int32_t* err_count, dr_stream_t stream);

/* ---------------------------------------------------------------------------
 * Accuracy metrics of top-k lists against test interactions, per user
 * (SURVEY.md §8f rank 1): precision@k (divrec/metrics/precision_at_k.py:6-22),
 * recall@k (recall_at_k.py:6-22), AP@k with the reference's formula
 * sum_p cumhits(p)/(p+1) / k (average_precision_at_k.py:6-24) and NDCG@k
 * (normalized_discounted_cumulative_gain.py:6-23). Positives as CSR: rowptr
 * int64 [n_users+1], items int32 sorted per row. Any output may be NULL.
 * recall is NaN for a user without positives (the reference divides by 0). */
int dr_rank_metrics(const void* recs, int rec_dtype, int64_t n_users, int k,
                    const int64_t* pos_rowptr, const int32_t* pos_items, float* precision,
                    float* recall, float* avg_precision, float* ndcg, dr_stream_t stream);

/* ---------------------------------------------------------------------------
 * Catalog histogram of recommendation lists: ADDS, for
 * every entry of recs [n_users, k] with 0 <= item < n_items, 1 to counts[item]
 * (int32 [n_items]) and its 0-based position to pos_sum[item] (uint64
 * [n_items], may be NULL). The caller zeroes both. Replaces the counting of
 * EntropyDiversityScore (divrec/metrics/entropy_diversity_score.py:19-26,
 * torch.unique counts) and PRI's avg_rank
 * (divrec/metrics/popularity_rank_correlation_for_items.py:28-39). Exact. */
int dr_catalog_histogram(const void* recs, int rec_dtype, int64_t n_users, int k,
                         int64_t n_items, int32_t* counts, uint64_t* pos_sum,
                         dr_stream_t stream);

/* ---------------------------------------------------------------------------
 * MMR diversity re-rank (config 5; no reference symbol — SURVEY.md §8a a16):
 * per user, greedily pick k_out of the C candidates maximising
 *   lambda * score_i - (1 - lambda) * max_{j in S} cos(e_i, e_j)
 * (ties -> lowest candidate position). cand_items int32 [n_users, C],
 * cand_scores fp32 [n_users, C], item_table bf16 [*, d]; out int32 [n_users, k_out]
 * (item ids in selection order). C <= 1024, k_out <= C, d in {64, 128}.
 * Candidate ids < 0 are empty slots; ids >= n_items are added to *err (int32
 * device counter, may be NULL) and never picked. A user left without live
 * candidates gets -1 for the remaining picks. n_items = 0 is DR_EINVAL.
 * Launch: one workgroup per CU looping over the users (the next user's
 * candidates are prefetched while one runs). */
int dr_mmr_rerank(const int32_t* cand_items, const float* cand_scores, int64_t n_users, int C,
                  const void* item_table, int64_t n_items, int d, int k_out, float lambda,
                  int32_t* out_items, int32_t* err, dr_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* DIVREC_HIP_H_ */
