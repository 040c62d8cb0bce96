/*
 * nais.h -- C-ABI of the MI355X-native NAIS scoring path (gfx950, libnais_hip.so).
 *
 * The reference (muyeon-jo/POI_recommendation_models) is pure Python + PyTorch and exposes no
 * FFI; the boundary this library replaces is the Python call surface of its NAIS hot path:
 *
 *   nais_forward        replaces NAIS_basic.forward            model.py:40-55  (+ attention_network :57-89)
 *                                NAIS_regionEmbedding.forward   model.py:132-142 (+ :144-180)
 *                                NAIS_region_distance_Embedding.forward model.py:231-244 (+ :246-297)
 *                                NAIS_distance_Embedding.forward model.py:340-353 (+ :355-395)
 *   nais_score_topk     replaces the per-user loop body of      validation.py:11-27 (NAIS_validation),
 *                                                               validation.py:38-55 (NAIS_region_validation),
 *                                                               validation.py:69-127 (NAIS_region_distance_validation,
 *                                                               also run with NAIS_distance_Embedding, run.py:431)
 *                       i.e. get_NAIS_batch_test* (batches.py:52-65, 110-139) + chunked forward + torch.topk
 *   nais_gather_rows    the embedding gather of model.py:64 (nn.Embedding -> index_select) as a standalone
 *                       HBM-roofline kernel
 *   nais_train_*        one NAIS_basic training step (run.py:91-109): train-mode forward with dropout
 *                       (model.py:22,40-89), backward of the attention pooling, dense embedding grads;
 *                       nais_adagrad* = torch.optim.Adagrad's update (run.py:89)
 *
 * Conventions: every pointer is caller-owned DEVICE memory (e.g. torch tensor.data_ptr()); the library
 * never allocates, frees or copies caller memory, never synchronises, and issues all work on `stream`
 * (a hipStream_t; NULL = legacy default stream). Calls are asynchronous and stream-ordered.
 * Scratch memory comes from a caller-supplied workspace sized by the matching *_workspace_size().
 * Return value: 0 on success, < 0 on error (see NAIS_E_*); nais_last_error() then describes it
 * (thread-local). All arithmetic is IEEE fp32 (fp64 for coordinates), as in the reference.
 */
#ifndef NAIS_H_
#define NAIS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NAIS_ABI_VERSION 14   /* 14: nais_pair_bound_topk / nais_pair_refine_topk take the optional per-entry table rows and per-slot history spans; 13: split16 pair tables, bounded gather + exact refine (nais_pair_table_split, nais_pair_bound_topk, nais_pair_refine_topk); 12: any embed_dim <= 256 and any hidden (generic-shape kernels); 11: hidden up to 256 (fp16x6 scoring, nais_forward), any variant on the x6n kernel */

/* model variants */
#define NAIS_VARIANT_BASIC 0           /* NAIS_basic                      model.py:8-97    */
#define NAIS_VARIANT_REGION 1          /* NAIS_regionEmbedding            model.py:99-187  */
#define NAIS_VARIANT_REGION_DISTANCE 2 /* NAIS_region_distance_Embedding  model.py:189-304 */
#define NAIS_VARIANT_DISTANCE 3        /* NAIS_distance_Embedding         model.py:306-408 */

/* arithmetic of the W1 x products in the catalog scorer (nais_score_topk / nais_score_catalog) */
#define NAIS_PRECISION_FP32 0          /* v_mfma_f32_32x32x2_f32: exact fp32 (k-ordered fmaf chain)           */
#define NAIS_PRECISION_FP16X3 1        /* v_mfma_f32_32x32x16_f16 on power-of-two-scaled hi/lo fp16 splits:
                                          3 products per fp32 product, fp32 accumulate, ~2^-21 relative;
                                          operands A_j = W1 diag(h_j) (split once per item) and t_c     */
#define NAIS_PRECISION_FP16X3_PAIRSPLIT 2 /* same arithmetic class, splitting x = h_j (.) t_c per pair
                                          (the reference's operand order; more VALU work)                 */
#define NAIS_PRECISION_FP16X6 3        /* fp32-faithful split (the default): hi/mid/lo fp16 pieces hold
                                          every operand exactly, 6 f16 MFMA products per fp32 product
                                          (dropped terms <= ~2^-33 relative, below fp32's 2^-24 product
                                          rounding), fp32 accumulate; item-side operands as FP16X3     */
#define NAIS_PRECISION_FP16X6_PAIRSPLIT 4 /* FP16X6 arithmetic on the per-pair split of x = h_j (.) t_c */

/* flags for nais_forward */
#define NAIS_FLAG_SIGMOID 1            /* apply sigmoid (model.py:55); else return the logits of attention_network */

/* error codes */
#define NAIS_OK 0
#define NAIS_E_INVALID (-1)            /* bad pointer / shape / dtype-implied size */
#define NAIS_E_UNSUPPORTED (-2)        /* a dimension outside the compiled kernel set */
#define NAIS_E_HIP (-3)                /* a HIP runtime error while launching */
#define NAIS_E_WORKSPACE (-4)          /* workspace missing or too small */

/*
 * Parameters of one NAIS model: device pointers to the reference's nn.Module parameters
 * (state_dict names in comments) plus their dimensions. Shapes (the reference builds
 * Linear(embed_size, hidden_size) for any sizes, model.py:9-38): embed_dim 1..256, hidden >= 1,
 * every entry point. The tuned kernels are compiled for embed_dim in {8, 16, 32, 64, 128} and
 * hidden <= 256 (scoring at precision FP16X6 with embed_dim 32 / 64 / 128, and nais_forward;
 * <= 128 for the other catalog precisions); every other shape runs the generic-shape kernels
 * (exact fp32 whatever the precision; nais_generic.hip) -- a caller with a width < 128 off that
 * set may instead zero-pad the tables (each half of the region variants' rows separately) and
 * attn_layer1's columns to the next native width for the tuned kernels (exact; the Python drop-in
 * does, model._NAISDevice._score_params). Training: the tuned / general kernels up to 128, the
 * generic-shape ones above. embed_dim > 256 is NAIS_E_UNSUPPORTED (the LDS budget).
 */
typedef struct nais_params {
  int32_t variant;              /* NAIS_VARIANT_* */
  int32_t embed_dim;            /* D: width of h_j (.) t (embed_size in every variant)                 */
  int32_t item_dim;             /* columns of embed_history/embed_target: D (basic, distance), D/2 (region*) */
  int32_t region_dim;           /* columns of embed_region: D/2 (region*), 0 (basic, distance)         */
  int32_t hidden;               /* H = attn_layer1.out_features (1..256, see above)                    */
  int32_t din;                  /* attn_layer1.in_features: D, or D+2 for region_distance / distance   */
  int64_t num_pois;             /* P = rows of embed_history / embed_target                            */
  int64_t num_regions;          /* R = rows of embed_region (0 for basic)                              */
  float beta;                   /* attention smoothing exponent (model.py:80), 0.5 in every driver     */
  int32_t precision;            /* NAIS_PRECISION_* (catalog scorer; nais_forward is always fp32)      */
  const float* embed_history;   /* embed_history.weight [P, item_dim]        model.py:15,106,198      */
  const float* embed_target;    /* embed_target.weight  [P, item_dim]        model.py:16,107,199      */
  const float* embed_region;    /* embed_region.weight  [R, region_dim]|NULL model.py:109,203         */
  const float* w1;              /* attn_layer1.weight   [H, din]             model.py:25,116,212      */
  const float* b1;              /* attn_layer1.bias     [H]                                           */
  const float* w2;              /* attn_layer2.weight   [1, H]               model.py:26,117,213      */
  const float* dist_w;          /* dist_layer.weight    [2, 2] | NULL        model.py:215             */
  const float* dist_b;          /* dist_layer.bias      [2]    | NULL                                 */
} nais_params_t;

/* Optional power-law geo prior blended into the catalog scores before the top-k (powerLaw.py:86-92,
 * run.py:55-59, run.py:537-539): G(u,c) = prod_j a*max(0.01, dist(coo_j, coo_c))^b (float64, history in
 * CSR order), G_norm = G / max_c G (unless the max is 0), score' = f32((1-alpha)*score) + alpha*G_norm
 * (float64), ranked on score'. out_scores then carries score' rounded to float32. */
typedef struct nais_prior {
  double a, b, alpha;
  const double* coords;         /* [P, 2] (lat, lng) float64 */
} nais_prior_t;

/* ABI version of the loaded library (== NAIS_ABI_VERSION it was built with). */
int32_t nais_abi_version(void);

/* Thread-local description of the last error returned by this thread. */
const char* nais_last_error(void);

/*
 * General forward (any per-row histories): for row r in [0,b) with history hist[r*hist_ld + j],
 * j in [0,n), and target item target[r], write out[r] = sigmoid(logit) (flags & NAIS_FLAG_SIGMOID)
 * or the logit of attention_network, exactly as model.py:57-89 (mask model.py:92-95, no
 * max-subtraction, beta-smoothed denominator). n == 0 gives logit 0.
 *   hist_region [b, n] (row stride hist_region_ld), target_region [b]: region variants only.
 *   target_lat_long [b, n, 2] f32 (row stride latlon_ld, in elements): region_distance and
 *   distance, = (|lat_c - lat_j|, |lng_c - lng_j|) as built at run.py:47-54 / validation.py:108-118;
 *   the kernels scale it x100 (model.py:265) or x1000 (distance, model.py:369) before dist_layer.
 *   nan_count (may be NULL): device int32, atomically incremented by the number of NaN logits
 *   (model.py:50-54 prints this count).
 */
int32_t nais_forward(const nais_params_t* params,
                     const int64_t* hist, int64_t b, int64_t n, int64_t hist_ld,
                     const int64_t* target,
                     const int64_t* hist_region, int64_t hist_region_ld,
                     const int64_t* target_region,
                     const float* target_lat_long, int64_t latlon_ld,
                     float* out, int32_t* nan_count, int32_t flags, void* stream);

/*
 * Full-catalog scoring + top-k for a list of users (validation.py:11-27 per-user body):
 * candidates of user u are every POI not in its training history
 *   indices[indptr[u] .. indptr[u+1])   (CSR of train_matrix, batches.py:55-56),
 * each scored with the variant's forward (sigmoid), then the k best are returned ordered by
 * (score desc, POI id asc); NaN ranks first (torch.topk semantics).
 *   users[i] (i < num_users): user ids to score; out_ids / out_scores are [num_users, k].
 *   region_of [P] int64: POI -> region (businessRegionEmbedList, run.py:149-152), region variants.
 *   coords [P, 2] float64 (lat, lng): (region_)distance -- (|dlat|, |dlng|) formed on the fly in
 *   float64, bit-identical to run.py:47-54. latlon_mat [P, P, 2] float64: the reference's own
 *   matrix (run.py:214), read instead when coords is NULL (feasible only for small P).
 *   k <= 1024 and every user needs at least k candidates (torch.topk raises otherwise; the
 *   caller checks -- the kernel writes id -1 / NaN for missing slots and counts them in *short_count).
 *   nan_count / short_count (device int32, may be NULL) are atomically incremented.
 */
size_t nais_score_topk_workspace_size(const nais_params_t* params, int32_t num_users, int32_t k,
                                      int32_t with_prior);
int32_t nais_score_topk(const nais_params_t* params,
                        const int64_t* indptr, const int64_t* indices,
                        const int32_t* users, int32_t num_users, int32_t k,
                        const int64_t* region_of, const double* coords,
                        const double* latlon_mat, const nais_prior_t* prior,
                        int32_t* out_ids, float* out_scores,
                        int32_t* nan_count, int32_t* short_count,
                        void* workspace, size_t workspace_bytes, void* stream);

/*
 * Scores only (the first half of nais_score_topk): scores[i * score_ld + c] = sigmoid score of POI c
 * for user users[i], c in [0, P); POIs in the user's history are written as -1.0f (they are not
 * candidates, batches.py:56). score_ld >= P. Used for parity tests and by callers that post-process
 * the full score row (e.g. the geo-prior blend).
 */
int32_t nais_score_catalog(const nais_params_t* params,
                           const int64_t* indptr, const int64_t* indices,
                           const int32_t* users, int32_t num_users,
                           const int64_t* region_of, const double* coords, const double* latlon_mat,
                           float* scores, int64_t score_ld, int32_t* nan_count, void* stream);

/*
 * Power-law prior rows (powerLaw.py:90-92): out[i * out_ld + c] = prod_j pr_d(dist(coo_j, coo_c)) for user
 * users[i], c in [0, P), float64 in the reference's operation order; history POIs get -1. out_max[i] =
 * max over the user's candidates (the normalize() divisor of run.py:55-59). coords [P, 2] float64.
 */
int32_t nais_powerlaw_prior(const double* coords, int64_t num_pois, const int64_t* indptr,
                            const int64_t* indices, const int32_t* users, int32_t num_users, double a,
                            double b, double* out, int64_t out_ld, double* out_max, void* stream);

/*
 * Pair-distance histogram for PowerLaw.fit_distance_distribution (powerLaw.py:41-55): hist[bin] = number of
 * pairs i < j within a user's history (all num_users users) with int(dist) == bin (km); pairs with
 * dist >= nbins or NaN are counted in *overflow. Both outputs are zeroed by the call.
 */
int32_t nais_distance_histogram(const double* coords, const int64_t* indptr, const int64_t* indices,
                                int64_t num_users, uint64_t* hist, int64_t nbins, uint64_t* overflow,
                                void* stream);

/*
 * Top-k of score rows (the second half of nais_score_topk): for row i in [0, num_rows), the k largest
 * entries of scores[i * score_ld + c], c in [0, P), ignoring negative entries (non-candidates), ordered
 * (score desc, c asc), NaN first -> out_ids / out_scores [num_rows, k]. k <= 1024.
 */
int32_t nais_topk_rows(const float* scores, int64_t score_ld, int64_t num_pois, int32_t num_rows,
                       int32_t k, int32_t* out_ids, float* out_scores, int32_t* short_count,
                       void* stream);

/*
 * Standalone embedding-row gather (model.py:64, nn.Embedding): out[i, :] = table[idx[i], :],
 * table [rows, dim] f32 row-major, idx [m] int64 (caller guarantees 0 <= idx < rows).
 */
int32_t nais_gather_rows(const float* table, int64_t rows, int32_t dim,
                         const int64_t* idx, int64_t m, float* out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * "Pairs" strategy of the full-catalog loop (validation.py:11-27). Every term of a user's score
 * for history item j and candidate c depends on (j, c) only (model.py:57-89), so a user list's
 * scores can be formed from two per-pair tables computed ONCE for the list's distinct history
 * items instead of once per user:
 *   nais_pair_rows     items[0 .. *num_items) = distinct history POIs of users[] (ascending),
 *                      rowmap[P] = row of each POI in items[] or -1. Workspace:
 *                      nais_pair_rows_workspace_size(P) bytes. *num_items is device memory.
 *   nais_pair_table    for item rows r < num_items and candidates c in [col0, col0 + cols):
 *                      e[r*ld + c-col0] = exp(a_rc) * [items[r] != c],  es[...] = e * (h_r . t_c),
 *                      with the catalog kernels' arithmetic for params->precision (split-fp16
 *                      where nais_score_catalog uses the fused split kernel, else exact fp32).
 *   nais_pair_gather   for every user and c in [col0, col0 + cols): N = sum_j es[row(j), c],
 *                      S = sum_j e[row(j), c] over the user's history in CSR order,
 *                      scores[slot*score_ld + c - score_col0] = sigmoid(N / S^beta) (history
 *                      POIs = -1, empty history = 0.5; score_col0 = the POI of column 0 of
 *                      scores, 0 for full rows); NaNs counted into *nan_count as
 *                      nais_score_catalog does.
 * The caller loops over column blocks sized to its memory budget and runs nais_topk_rows.
 *   work (nais_pair_table, nais_pair_gather_topk; may be NULL): one int32 of device memory private
 *                      to the stream. Given, the launch runs as a work queue -- about one
 *                      resident round of workgroups takes (item group, column tile) or user slots
 *                      from this counter (zeroed by the call, stream-ordered) until they run out,
 *                      so a CU-masked stream whose CU count is not a multiple of the shader-engine
 *                      count still uses every CU (nais_pair_table: the 16x16x32 fp16x6 kernel
 *                      only; other shapes ignore it). Results are identical either way.
 *   nais_pair_gather_topk  the same sums and scores, but instead of score rows each user keeps a
 *                      running top-k: keys[slot*k ..] (uint64, sorted descending, kcount[slot]
 *                      valid; zero kcount before the first call) with key = ordered(score) << 32 |
 *                      (0xFFFFFFFF - poi), i.e. torch.topk's (score desc) with ties by POI id asc
 *                      and NaN first; history POIs are never candidates. Columns of one call may
 *                      be any block; the calls of one user list must be stream-ordered. k <= 256.
 *   nais_topk_keys_finish  keys -> out_ids / out_scores [num_users, k] (short lists padded with
 *                      -1 / NaN and counted into *short_count), as nais_topk_rows reports them.
 */
size_t nais_pair_rows_workspace_size(int64_t num_pois);
int32_t nais_pair_rows(const int64_t* indptr, const int64_t* indices, const int32_t* users,
                       int32_t num_users, int64_t num_pois, int32_t* rowmap, int64_t* items,
                       int64_t* num_items, void* workspace, size_t workspace_bytes, void* stream);
int32_t nais_pair_table(const nais_params_t* params, const int64_t* items, int64_t num_items,
                        int64_t col0, int64_t cols, const int64_t* region_of,
                        const double* coords, const double* latlon_mat, float* e, float* es,
                        int64_t ld, int32_t* work, void* stream);
int32_t nais_pair_gather(const float* e, const float* es, int64_t ld, const int32_t* rowmap,
                         const int64_t* indptr, const int64_t* indices, const int32_t* users,
                         int32_t num_users, int64_t col0, int64_t cols, float beta, float* scores,
                         int64_t score_ld, int64_t score_col0, int32_t* nan_count, void* stream);
int32_t nais_pair_gather_topk(const float* e, const float* es, int64_t ld, const int32_t* rowmap,
                              const int64_t* indptr, const int64_t* indices, const int32_t* users,
                              int32_t num_users, int64_t col0, int64_t cols, float beta, int32_t k,
                              uint64_t* keys, int32_t* kcount, int32_t* nan_count, int32_t* work,
                              void* stream);
int32_t nais_topk_keys_finish(const uint64_t* keys, const int32_t* kcount, int32_t num_users, int32_t k,
                              int32_t* out_ids, float* out_scores, int32_t* short_count, void* stream);
/*
 * Bounded gather + exact refine (filter-and-refine top-k; DESIGN.md (d) "bounded gather"): the
 * lists of nais_pair_gather_topk -- the same ids and score bits -- from half the gathered bytes.
 *   nais_pair_table_split  nais_pair_table's pairs stored split16: hi[r*ld + c-col0] = (top 16 bits
 *                      of e*s) << 16 | (top 16 bits of e) -- both values truncated to 8 significant
 *                      bits -- and ex[2*(r*ld + c-col0)] = e, ex[... + 1] = e*s (the exact pair,
 *                      8 bytes side by side; ex row pitch 2*ld).
 *   nais_pair_bound_topk   per column block (stream-ordered over the blocks of one user list): each
 *                      user's S, N = sum over its history of the truncated e, e*s and sum |e*s| give
 *                      an interval around every candidate's exact score (the fp32 arithmetic of
 *                      nais_pair_gather_topk on the untruncated pairs); lo_keys[slot*k ..] / lo_count
 *                      keep the k best lower bounds (zero lo_count before the first block), and the
 *                      key (upper bound, id) of every candidate whose upper bound reaches the k-th
 *                      lower bound so far is appended to surv[slot*surv_cap ..] (surv_count[slot];
 *                      zero it before the first block; compacted when full, -1 if it overflows).
 *                      Keys as nais_pair_gather_topk. ld % 4 == 0, hi 16-byte aligned, k <= 256.
 *   nais_pair_refine_topk  after the last block: for each survivor whose upper key reaches the final
 *                      k-th lower key (every column for an overflowed user), the exact N, S from the
 *                      ex pairs in history (CSR) order and its score; keys / kcount receive the top-k
 *                      exactly as nais_pair_gather_topk leaves them (NaNs counted into *nan_count).
 *                      ex: block b (columns col0 + b*block_cols ..) at ex + b*block_stride (uint32
 *                      words, even), rows of ld pairs (nais_pair_table_split's ex). stats (may be
 *                      NULL): stats[0] += candidates refined, stats[1] += overflowed users. tau (may
 *                      be NULL): per user a threshold key to use when larger than its own k-th lower
 *                      key -- a column shard of a process group passes the k-th lower key over ALL
 *                      shards (exchanged after the last block) and then returns only its candidates
 *                      that can reach the global top-k: kcount may be < k (padding as short lists).
 *                      A column shard's k-th lower key is a lower bound of the global k-th exact key,
 *                      so every global winner on this shard is still returned.
 *   entry_rows (both; may be NULL): entry_rows[e] = rowmap[indices[e]] for every CSR entry e of the
 *                      listed users -- the table row of each history entry, read beside its POI id
 *                      instead of after it. spans (nais_pair_bound_topk; may be NULL):
 *                      spans[2*s] = indptr[users[s]], spans[2*s+1] = the history length of users[s]
 *                      -- one load per slot instead of two in a row. Both only shorten the chains
 *                      of dependent loads (ABI 14); the results are the same with or without them.
 */
int32_t nais_pair_table_split(const nais_params_t* params, const int64_t* items, int64_t num_items,
                              int64_t col0, int64_t cols, const int64_t* region_of,
                              const double* coords, const double* latlon_mat, uint32_t* hi,
                              uint32_t* ex, int64_t ld, int32_t* work, void* stream);
int32_t nais_pair_bound_topk(const uint32_t* hi, int64_t ld, const int32_t* rowmap,
                             const int64_t* indptr, const int64_t* indices, const int32_t* users,
                             int32_t num_users, int64_t col0, int64_t cols, float beta, int32_t k,
                             uint64_t* lo_keys, int32_t* lo_count, uint64_t* surv, int32_t* surv_count,
                             int32_t surv_cap, const int32_t* entry_rows, const int64_t* spans,
                             int32_t* work, void* stream);
int32_t nais_pair_refine_topk(const uint32_t* ex, int64_t block_stride,
                              int64_t ld, int64_t block_cols, const int32_t* rowmap,
                              const int64_t* indptr, const int64_t* indices, const int32_t* users,
                              int32_t num_users, int64_t col0, int64_t cols, float beta, int32_t k,
                              const uint64_t* lo_keys, const int32_t* lo_count, const uint64_t* surv,
                              const int32_t* surv_count, int32_t surv_cap, const uint64_t* tau,
                              uint64_t* keys, int32_t* kcount, int32_t* nan_count, int32_t* stats,
                              const int32_t* entry_rows, void* stream);
/*
 * Power-law prior on the pairs route (powerLaw.py:86-92, run.py:537-539; the direct route's
 * nais_score_topk with a prior computes the same G rows per user):
 *   nais_pair_prior_table   pr[r*ld + c-col0] = pr_d(dist(items[r], c)) (float64, powerLaw.py's
 *                           operation order) for r < num_items, c in [col0, col0 + cols).
 *   nais_pair_prior_gather  per user slot and c in [col0, col0 + cols):
 *                           g[slot*g_ld + c-g_col0] = prod_j pr[row(j), c] over the history in CSR
 *                           order (1.0 for an empty history; -1.0 for history POIs) -- the bits of
 *                           nais_powerlaw_prior -- and gmax_bits[slot] = max(gmax_bits[slot], the
 *                           block's largest candidate value) as u64 bits; zero gmax_bits before the
 *                           first block. ld must be a multiple of 4 (32-byte loads).
 *   nais_topk_blend_rows    top-k of f32((1 - alpha) * score) + alpha * g / gmax (float64; history
 *                           POIs, score < 0, excluded) per row, (score desc, id asc), as
 *                           nais_score_topk ranks with a prior; out_scores = the blended score as f32.
 *   nais_topk_blend_rows_f64  the same, and (out_blend != NULL) the f64 blended score of every
 *                           returned candidate (NaN for padding) -- the key a column-sharded job
 *                           merges on.
 *   nais_topk_merge_f64     merge of per-column-block lists: row r's m candidates
 *                           (keys[r*m + i] f64, ids[r*m + i] global POI ids, id < 0 = padding) ->
 *                           the k best by (key desc, id asc), NaN first, as out_ids / out_scores
 *                           (f32) / out_keys (f64, optional). m <= 2048, k <= m.
 */
int32_t nais_pair_prior_table(const double* coords, int64_t num_pois, const int64_t* items,
                              int64_t num_items, int64_t col0, int64_t cols, double a, double b,
                              double* pr, int64_t ld, void* stream);
#define NAIS_PRIOR_FINITE 1   /* flags: every pr entry is finite and >= +0 (a > 0, a * max(0.01, d)^b
                                 finite for every distance): a product that underflowed to +0.0
                                 stays +0.0, so
                                 the gather stops reading a wave's rows once all its columns are 0 */
int32_t nais_pair_prior_gather(const double* pr, int64_t ld, const int32_t* rowmap,
                               const int64_t* indptr, const int64_t* indices, const int32_t* users,
                               int32_t num_users, int64_t col0, int64_t cols, double* g, int64_t g_ld,
                               int64_t g_col0, uint64_t* gmax_bits, int32_t flags, void* stream);
int32_t nais_topk_blend_rows(const float* scores, int64_t score_ld, const double* g, int64_t g_ld,
                             const uint64_t* gmax_bits, int64_t num_pois, int32_t num_rows, int32_t k,
                             double alpha, int32_t* out_ids, float* out_scores, int32_t* short_count,
                             void* stream);
int32_t nais_topk_blend_rows_f64(const float* scores, int64_t score_ld, const double* g, int64_t g_ld,
                                 const uint64_t* gmax_bits, int64_t num_pois, int32_t num_rows, int32_t k,
                                 double alpha, int32_t* out_ids, float* out_scores, double* out_blend,
                                 int32_t* short_count, void* stream);
int32_t nais_topk_merge_f64(const double* keys, const int64_t* ids, int32_t num_rows, int32_t m,
                            int32_t k, int64_t* out_ids, float* out_scores, double* out_keys,
                            void* stream);

/*
 * A stream restricted to the CUs whose bits are set in cu_mask[mask_words] (bit i = CU i), for
 * running an MFMA-bound and an HBM-bound kernel side by side on disjoint CUs (the pairs strategy's
 * table / gather overlap). Destroy with nais_stream_destroy.
 */
int32_t nais_stream_create_cu_mask(const uint32_t* cu_mask, uint32_t mask_words, void** stream);
int32_t nais_stream_destroy(void* stream);

/*
 * New4 family (model.py:1169-1306): the per-POI context tables its forward builds
 * from the near-POI lists before NAIS_basic's attention (self_attention, model.py:1272-1295):
 *   ext_history[p] = [embed_history[p] | result_in[p] | result_out[p]]   [P, embed_size]
 *   ext_target[p]  = [embed_target[p]  | result_out[p] | result_in[p]]   [P, embed_size]
 * embed_history / embed_target [P, embed_size/2], embed_ingoing / embed_outgoing [P, embed_size/4],
 * near_pois [P, num_near] int64 (nearPOI, datasets.py:418). Scoring New4 is then the basic variant
 * (nais_forward / nais_score_topk) with these two tables as embed_history / embed_target.
 */
int32_t nais_new4_tables(const float* embed_history, const float* embed_target,
                         const float* embed_ingoing, const float* embed_outgoing,
                         int64_t num_pois, int32_t embed_size, const int64_t* near_pois,
                         int32_t num_near, float* ext_history, float* ext_target, void* stream);

/*
 * The near-POI pooling every table-based New4-family member runs (New4 / New4_padding /
 * all_in_out / transform_ingoing_outgoing / transform_attn: two pools, model.py:1269-1295,
 * 1551-1566, 1922-1950; nearPOI_embedding / only_area_not_inout: one pool, model.py:1680-1686,
 * 2198-2218; no_POI_emb: two pools of width embed_size/2, model.py:1797-1812). For every p < P:
 *   x_k = kv_src[near[p][k]], q = query_src[near[p][0]]              (rows of width dim)
 *   key_k = wk x_k + bk, val_k = wv x_k + bv, q = wq q + bq         (nn.Linear [dim, dim], [dim];
 *                                                 NULL weight = identity, NULL bias = zero)
 *   out[p * out_ld + c] = (softmax(q . reshape(key, [dim, K]) / sqrt(scale_dim)) @ val)[c]
 * out may point into a column range of a wider row table (out_ld >= dim).
 * nais_copy_columns: dst[p * dst_ld + dst_col0 + c] = src[p * src_ld + c], p < rows, c < dim.
 */
int32_t nais_near_attention(const float* query_src, const float* kv_src, int64_t num_pois,
                            int32_t dim, const int64_t* near_pois, int32_t num_near,
                            const float* wq, const float* bq, const float* wk, const float* bk,
                            const float* wv, const float* bv, float scale_dim, float* out,
                            int64_t out_ld, void* stream);
int32_t nais_copy_columns(const float* src, int64_t src_ld, int64_t rows, int32_t dim, float* dst,
                          int64_t dst_ld, int32_t dst_col0, void* stream);

/*
 * transform_attn (model.py:1959-2098): dot-product attention over New4-layout rows (SURVEY.md
 * 8(f4)). Its query/key/value projections act on one POI row each, so they are per-POI tables:
 *   xh, xt   [P, D]  history / target rows (nais_near_attention + nais_copy_columns, New4 layout)
 *   qt = xt Wq^T + bq, kh = xh Wk^T + bk, vh = xh Wv^T + bv   [P, D]   (nais_linear_rows)
 * and the prediction (model.py:2030-2055) is
 *   logit = sum_j m_j e_j (vh_j . xt_c) / (sum_j m_j e_j)^beta,  e_j = exp(qt_c . kh_j / sqrt(scale_dim))
 * with m_j = [h_j != c]; scale_dim = embed_size (torch.sqrt(torch.tensor(self.embed_size))).
 * nais_dot_forward: out[r] for rows r < b as nais_forward (flags, nan_count). For n == 1 it
 *   restates the reference's shapes exactly: exp_A.squeeze(dim=-1) (model.py:2042) leaves [b] and
 *   the mask broadcast couples all b rows: out_r = m_r s_r S / (m_r S)^beta, S = sum_r' e_r'.
 * nais_dot_pair_table: the pair tables of nais_pair_table for this core (E = e_jc, ES = e_jc s_jc),
 *   consumed by nais_pair_gather unchanged.
 * nais_dot_single_fixup: for the listed users with exactly one history item, overwrite their score
 *   rows with new4_validation's chunk-coupled scores (1024-candidate chunks of the ascending
 *   complement list, validation.py:262-270): score_c = sigmoid(s_c S_k / S_k^beta), S_k the sum of
 *   e over c's chunk. Columns [col0, col0 + cols) of rows laid out as in nais_pair_gather.
 * nais_linear_rows: y[r, :dout] = x[r, :din] W^T + b (nn.Linear; b may be NULL), dout <= 256.
 */
typedef struct nais_dot_tables {
  int32_t embed_dim;            /* D (<= 128)                                                 */
  int64_t num_pois;             /* P                                                          */
  float beta;                   /* 0.5                                                        */
  float scale_dim;              /* logits divide by sqrt(scale_dim) (= embed_size)            */
  const float* xh;              /* [P, D] each                                                */
  const float* xt;
  const float* qt;
  const float* kh;
  const float* vh;
} nais_dot_tables_t;

int32_t nais_linear_rows(const float* x, int64_t x_ld, int64_t rows, int32_t din, const float* w,
                         const float* b, int32_t dout, float* y, int64_t y_ld, void* stream);
int32_t nais_dot_forward(const nais_dot_tables_t* tables, const int64_t* hist, int64_t b, int64_t n,
                         int64_t hist_ld, const int64_t* target, float* out, int32_t* nan_count,
                         int32_t flags, void* stream);
int32_t nais_dot_pair_table(const nais_dot_tables_t* tables, const int64_t* items, int64_t num_items,
                            int64_t col0, int64_t cols, float* e, float* es, int64_t ld,
                            void* stream);
int32_t nais_dot_single_fixup(const nais_dot_tables_t* tables, const int64_t* indptr,
                              const int64_t* indices, const int32_t* users, int64_t num_users,
                              int64_t col0, int64_t cols, float* scores, int64_t score_ld,
                              int64_t score_col0, void* stream);

/*
 * NAIS_region_distance_disentangled_Embedding (model.py:409-541): two attention
 * MLPs (POI rows and region rows, both embed_size wide) with a shared additive distance term
 * d_j = sum_e embed_distance[0][e] * target_distance[r, j]; forward (model.py:446-455) =
 *   sigmoid( sum_j a_j (h_j . t) + rho_j (g_j . g_t) ),
 *   a_j = m_j exp(l_j + d_j) / (sum m exp(l + d))^beta, rho_j likewise with the region MLP.
 * Arguments as nais_forward (regions per entry / per row, target_distance [b, n] f32 with row
 * stride dist_ld = run.py:326-333's target_dist). Eval arithmetic (the model has no dropout).
 * nais_pair_distances: out[r * n + j] = f32(powerLaw.dist(coords[target[r]], coords[hist[j]]))
 *   (haversine km, float64 in the reference's order) -- run.py:326-333 for one batch (one shared
 *   history of n items, b targets); coords [P, 2] (lat, lng) float64.
 * The reference's evaluation call for this model (run.py:353) does not match
 * NAIS_region_distance_validation's signature, so only the forward has a defined meaning.
 */
typedef struct nais_disent_params {
  int32_t embed_dim;            /* D (<= 128)                                                 */
  int32_t hidden;               /* H (<= 128)                                                 */
  int64_t num_pois, num_regions;
  float beta;
  const float* embed_history;   /* [P, D]                                                     */
  const float* embed_target;    /* [P, D]                                                     */
  const float* embed_region;    /* [R, D]                                                     */
  const float* embed_distance;  /* [dist_embed_size, D] (row 0 is read)                       */
  const float* w1;              /* attn_layer1 [H, D], [H]; attn_layer2 [1, H]                */
  const float* b1;
  const float* w2;
  const float* region_w1;       /* region_attn_layer1 [H, D], [H]; region_attn_layer2 [1, H]  */
  const float* region_b1;
  const float* region_w2;
} nais_disent_params_t;

int32_t nais_disent_forward(const nais_disent_params_t* params, const int64_t* hist, int64_t b,
                            int64_t n, int64_t hist_ld, const int64_t* target,
                            const int64_t* hist_region, int64_t hist_region_ld,
                            const int64_t* target_region, const float* target_distance,
                            int64_t dist_ld, float* out, int32_t* nan_count, int32_t flags,
                            void* stream);
int32_t nais_pair_distances(const double* coords, const int64_t* hist, int64_t n,
                            const int64_t* target, int64_t b, float* out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Training step of NAIS_basic on one get_NAIS_batch batch (batches.py:24-50):
 * b rows (target[b], int64 POI ids) that all share ONE history hist[n] (int64, the user's positives;
 * the reference repeats it b times, batches.py:30). Replaces, for this batch shape,
 *   prediction = model(user_history, train_data)   (run.py:103; model.py:40-89 in train mode)
 *   loss.backward()                                (run.py:105; BCELoss model.py:21)
 * NAIS_VARIANT_BASIC; embed_dim up to 256, any hidden (fused MFMA kernels at embed_dim in
 * {8,16,32,64}, hidden <= 64; a general kernel up to 128; the generic-shape kernels above -- see
 * nais_train_forward_ex for the region variants).
 *
 * Dropout (nn.Dropout(dropout_p), model.py:22,71) keeps hidden unit i of pair (row c, item j) iff
 * a counter hash of (seed, c*n + j, i) is >= dropout_p * 2^32 and scales kept units by 1/(1-p);
 * dropout_p = 0 is eval-mode arithmetic. nais_dropout_mask() materialises the same mask
 * (uint8 [b, n, hidden], 1 = kept) for tests.
 *
 * nais_train_forward: pred[b] = sigmoid(logit) (model.py:55); saved[2b] = (S, N) per row for the
 *   backward; optional nan_count (+= rows whose logit is NaN, model.py:50-54).
 * nais_train_backward: given grad_pred[b] = dL/dpred (e.g. from BCELoss's backward), ADDS the
 *   gradients into grad_embed_history / grad_embed_target ([num_pois, embed_dim], dense, rows by
 *   POI id; repeated ids are summed with fp32 atomics), grad_w1 [hidden, embed_dim], grad_b1
 *   [hidden], grad_w2 [hidden]. Same params, hist, target, dropout_p and seed as the forward.
 *   Both calls take a workspace of nais_train_workspace_size(params, b, n) bytes (the forward's
 *   may be reused by the backward once the forward has run).
 * -------------------------------------------------------------------------------------------- */
size_t nais_train_workspace_size(const nais_params_t* params, int64_t b, int64_t n);

int32_t nais_train_forward(const nais_params_t* params, const int64_t* hist, int64_t n,
                           const int64_t* target, int64_t b, float dropout_p, uint64_t seed,
                           float* pred, float* saved, int32_t* nan_count, void* workspace,
                           size_t workspace_bytes, void* stream);

int32_t nais_train_backward(const nais_params_t* params, const int64_t* hist, int64_t n,
                            const int64_t* target, int64_t b, float dropout_p, uint64_t seed,
                            const float* pred, const float* saved, const float* grad_pred,
                            float* grad_embed_history, float* grad_embed_target, float* grad_w1,
                            float* grad_b1, float* grad_w2, void* workspace,
                            size_t workspace_bytes, void* stream);

int32_t nais_dropout_mask(uint64_t seed, int64_t b, int64_t n, int32_t hidden, float dropout_p,
                          uint8_t* out, void* stream);

/*
 * The same training forward / backward for every NAIS variant (NAIS_basic, NAIS_regionEmbedding,
 * NAIS_region_distance_Embedding, NAIS_distance_Embedding; run.py:91-280, 365-430) and any
 * embed_dim / hidden up to 128 (run.py's
 * defaults are factor_num = hidden_dim = 128). NAIS_basic at embed_dim in {8,16,32,64}, hidden <= 64
 * runs the fused MFMA kernels above; everything else a general kernel with the same math and the
 * same dropout draws. The region variants read full rows [embed_history | embed_region[region]]:
 *   side->hist_region [n], side->target_region [b]  (regions of the history items / target rows,
 *   get_NAIS_batch_region, batches.py:67-108); region_distance also side->target_lat_long
 *   [b, n, 2] f32, row stride latlon_ld (run.py:240-245), x100 before dist_layer (model.py:265).
 * NAIS_distance_Embedding reads basic rows and side->target_lat_long (x1000, model.py:369).
 * The two distance variants have no dropout (model.py:268, 369-371): pass dropout_p = 0.
 * Gradients are ADDED into grads (dense, fp32 atomics for repeated ids); embed_region and
 * dist_w / dist_b are required for the variants that have them. nais_train_forward / _backward
 * above are these with side = NULL (NAIS_basic only). Workspace: nais_train_workspace_size().
 */
typedef struct nais_train_side {
  const int64_t* hist_region;     /* [n]                                                        */
  const int64_t* target_region;   /* [b]                                                        */
  const float* target_lat_long;   /* [b, n, 2] f32 (region_distance)                           */
  int64_t latlon_ld;              /* row stride of target_lat_long in elements (>= 2n)         */
  /* optional u cache (general kernels, nais_train_ucache_size() > 0): with ucache_bytes >= that
   * size, nais_train_forward_ex leaves every pair's post-dropout W1 x + b1, h . t and attention
   * logit here and nais_train_backward_ex of the SAME batch, parameters and seed reads them instead
   * of recomputing the forward (a third of its MFMA work); NULL = recompute */
  float* ucache;
  uint64_t ucache_bytes;
} nais_train_side_t;

/* Bytes of the u cache for (params, b, n): 0 where the fused kernels run (they keep no cache) or
 * above 1 GiB (the backward then recomputes). */
size_t nais_train_ucache_size(const nais_params_t* params, int64_t b, int64_t n);

typedef struct nais_train_grads {
  float* embed_history;           /* [P, item_dim]  */
  float* embed_target;            /* [P, item_dim]  */
  float* embed_region;            /* [R, region_dim] (region variants)                          */
  float* w1;                      /* [H, din]       */
  float* b1;                      /* [H]            */
  float* w2;                      /* [H]            */
  float* dist_w;                  /* [2, 2] (region_distance)                                   */
  float* dist_b;                  /* [2]            */
} nais_train_grads_t;

int32_t nais_train_forward_ex(const nais_params_t* params, const nais_train_side_t* side,
                              const int64_t* hist, int64_t n, const int64_t* target, int64_t b,
                              float dropout_p, uint64_t seed, float* pred, float* saved,
                              int32_t* nan_count, void* workspace, size_t workspace_bytes,
                              void* stream);
int32_t nais_train_backward_ex(const nais_params_t* params, const nais_train_side_t* side,
                               const int64_t* hist, int64_t n, const int64_t* target, int64_t b,
                               float dropout_p, uint64_t seed, const float* pred,
                               const float* saved, const float* grad_pred,
                               const nais_train_grads_t* grads, void* workspace,
                               size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused training step of NAIS_basic (run.py:101-109 in one call; embed_dim / hidden up to 128,
 * the fused MFMA kernels where they apply, else the general ones): forward, BCELoss (model.py:21) added into
 * *loss_sum (device float, mean over the b rows -- run.py's train_loss accumulates loss.item()),
 * backward, and torch.optim.Adagrad's update of all five parameters IN PLACE (the params pointers
 * are written). Adagrad state lives in nais_adagrad_state_t; its gradient scratch must be all zero
 * on entry and is left all zero. Rows with a NaN prediction (a single-item history equal to its
 * target, model.py:92-95) are counted into *bad_rows (device int32); while *bad_rows != 0 the
 * update is skipped (the reference's BCELoss raises on such a batch). pred [b] is optional.
 * Workspace: nais_train_step_workspace_size(params, b, n) bytes.
 * -------------------------------------------------------------------------------------------- */
typedef struct nais_adagrad_state {
  float lr, lr_decay, weight_decay, eps;   /* torch.optim.Adagrad arguments (run.py:89)            */
  int64_t step;                            /* step count including this one (torch state['step']) */
  float* sum_embed_history;                /* Adagrad accumulators, shapes of the parameters       */
  float* sum_embed_target;
  float* sum_w1;
  float* sum_b1;
  float* sum_w2;
  float* grad_embed_history;               /* [P, D] zero-maintained gradient scratch              */
  float* grad_embed_target;                /* [P, D]                                               */
  float* grad_small;                       /* [H*din + 2H]: w1 | b1 | w2                           */
  int32_t* stamp_embed_history;            /* [P] row-claim stamps, initialised to 0               */
  int32_t* stamp_embed_target;             /* [P]                                                  */
} nais_adagrad_state_t;

size_t nais_train_step_workspace_size(const nais_params_t* params, int64_t b, int64_t n);

int32_t nais_train_step(const nais_params_t* params, const nais_adagrad_state_t* opt,
                        const int64_t* hist, int64_t n, const int64_t* target, const float* labels,
                        int64_t b, float dropout_p, uint64_t seed, float* loss_sum,
                        int32_t* bad_rows, float* pred, void* workspace, size_t workspace_bytes,
                        void* stream);

/*
 * The same fused step for the region / distance variants (run.py:139-200 NAIS_regionEmbedding,
 * :206-262 NAIS_region_distance_Embedding, :365-430 NAIS_distance_Embedding; batches from
 * get_NAIS_batch_region, batches.py:67-108): side = the batch's region ids / target_lat_long as
 * for nais_train_forward_ex (its ucache fields are ignored: the step keeps its own in the
 * workspace). opt covers embed_history / embed_target (rows of item_dim floats), attn_layer1 (its
 * grad_small block is [hidden * din | hidden | hidden]) and attn_layer2; opt_side the variant's
 * extra parameters, updated densely (torch.optim.Adagrad over model.parameters(), run.py:155):
 * embed_region [num_regions, region_dim] and / or dist_layer (weight [2, 2], bias [2]), each with
 * a zero-maintained gradient scratch. NAIS_basic with side = opt_side = NULL is nais_train_step.
 */
typedef struct nais_adagrad_side {
  float* sum_embed_region;                 /* [num_regions, region_dim] (region variants)          */
  float* grad_embed_region;                /* same shape, zero-maintained                          */
  float* sum_dist_w;                       /* [4] (distance variants)                              */
  float* sum_dist_b;                       /* [2]                                                  */
  float* grad_dist;                        /* [6]: dist_w | dist_b, zero-maintained                */
} nais_adagrad_side_t;

int32_t nais_train_step_ex(const nais_params_t* params, const nais_train_side_t* side,
                           const nais_adagrad_state_t* opt, const nais_adagrad_side_t* opt_side,
                           const int64_t* hist, int64_t n, const int64_t* target, const float* labels,
                           int64_t b, float dropout_p, uint64_t seed, float* loss_sum,
                           int32_t* bad_rows, float* pred, void* workspace, size_t workspace_bytes,
                           void* stream);

/*
 * get_NAIS_batch (batches.py:24-50) for one user on the device: hist [n] = the
 * user's n = indptr[user+1]-indptr[user] positives (CSR rows sorted ascending) in a seeded random
 * order; target / labels [n * (1 + num_ng)] = rows [pos_i, neg_i1 .. neg_i,num_ng], labels 1 / 0.
 * Negatives: distinct, uniform over the POIs not in the history (the reference's shuffle-and-slice
 * distribution; not Python's random stream). *err (optional) is set to 1 if n disagrees with indptr.
 */
int32_t nais_make_train_batch(const int64_t* indptr, const int64_t* indices, int64_t user,
                              int64_t n, int64_t num_pois, int32_t num_ng, uint64_t seed,
                              int64_t* hist, int64_t* target, float* labels, int32_t* err,
                              void* stream);

/*
 * torch.optim.Adagrad's update (run.py:89; lr_decay folded into clr = lr / (1 + (step-1) lr_decay)):
 *   g' = g + weight_decay * p ; state += g' * g' ; p -= clr * g' / (sqrt(state) + eps)
 * nais_adagrad: every element of a tensor of numel floats.
 * nais_adagrad_rows: only rows[num_rows] of a [*, dim] tensor, weight_decay 0. Rows whose
 *   gradient is zero are left bit-identical by the dense update, so this equals nais_adagrad
 *   when `rows` covers every row with a nonzero gradient. Rows are distinct, or sorted with
 *   repeats: an entry equal to the one before it is skipped (each row updated once).
 */
int32_t nais_adagrad(float* param, float* state_sum, const float* grad, int64_t numel, float clr,
                     float weight_decay, float eps, void* stream);
int32_t nais_adagrad_rows(float* param, float* state_sum, const float* grad, int32_t dim,
                          const int64_t* rows, int64_t num_rows, float clr, float eps,
                          void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NAIS_H_ */
