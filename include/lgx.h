/*
 * lgx.h -- C ABI of liblgx.so, the MI355X (gfx950) LightGCN propagation + scoring engine.
 *
 * Conventions
 *   - extern "C", plain pointers and sizes, no torch / no C++ types.
 *   - Every data pointer is caller-owned DEVICE memory unless the name ends in `_host`.
 *     The library never allocates on a compute call: scratch is passed in as `ws` / `ws_bytes`
 *     sized by the matching *_workspace() query.
 *   - Every call is stream-ordered on `stream` (a hipStream_t; NULL = the legacy default stream)
 *     and never synchronises the host, so it can be captured into a hipGraph.
 *   - Return value: LGX_OK (0) or an LGX_ERR_* code; lgx_last_error() returns a thread-local
 *     message for the last failing call on this thread.  No C++ exception crosses the ABI.
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   lgx_build_norm_adj     Loader.getSparseGraph build branch  lightGCN/LightGCN-PyTorch-master/code/dataloader.py:339-376
 *                          Data.get_adj_mat pre_adj branch      LightGCN-tf/utility/load_data.py:91-104
 *   lgx_csr_from_coo_rows  _convert_sp_mat_to_sp_tensor + coalesce (dataloader.py:331-337,373-374)
 *   lgx_propagate_layer /  LightGCN.computer()                  code/model.py:145-177 (torch.sparse.mm :171)
 *   lgx_propagate          TF _create_lightgcn_embed            LightGCN-tf/LightGCN.py:232-253
 *   lgx_spmm_csr           torch.sparse.mm(G, X) (forward, and the backward G^T dY = G dY)  model.py:171
 *   lgx_score_dense        LightGCN.getUsersRating              code/model.py:179-184; TF batch_ratings LightGCN.py:148
 *   lgx_score_topk         Procedure.Test mask + torch.topk     code/Procedure.py:127-135;
 *                          batch_test.test mask + evaluator     LightGCN-tf/utility/batch_test.py:47-70
 *                          recommend.py global min/max          recommend.py:163-164, 375-377
 *   lgx_score_minmax       np.max / np.min of the U x I dot     recommend.py:163-164, 377; utils.py:500-529
 *   lgx_topk_rows          c_top_k_array_index                  LightGCN-tf/evaluator/cpp/include/tools.h:13-33
 *   lgx_foldout_metrics    evaluate_foldout                     LightGCN-tf/evaluator/cpp/include/evaluate_foldout.h:115-195
 *   lgx_test_metrics       Procedure.Test metric sums           lightGCN/LightGCN-PyTorch-master/code/Procedure.py:60-72
 *   lgx_gather_scores      accuracy_cf / elasticity_item per-user candidate dot  recommend.py:167-171, 214-217
 *   lgx_parse_lines_*      Loader / Data file parsing            code/dataloader.py:247-277; load_data.py:27-48
 *   lgx_strat_labels/select create_candidates_stratification   recommend.py:314-452
 *   lgx_sample_bpr         sample_negative / sample_negative_ByUser   sources/sampling.cpp:27-86
 *   lgx_bpr_loss_*         LightGCN.bpr_loss + its backward        code/model.py:196-209; utils.py:43-52
 *   lgx_adam_step          BPRLoss's torch.optim.Adam step          code/utils.py:41,50
 *   lgx_list_dot_reduce    difference / ser1 / ser2 / diversity per-user list products
 *                          recommend.py:305-307; utils.py:34-35, 117-121, 265-267
 */
#ifndef LGX_H
#define LGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* lgx_stream_t; /* == hipStream_t */

#define LGX_OK 0
#define LGX_ERR_INVALID_ARG 1
#define LGX_ERR_HIP 2
#define LGX_ERR_UNSUPPORTED 3
#define LGX_ERR_WORKSPACE 4

#define LGX_DTYPE_F32 0  /* fp32 storage, fp32 arithmetic */
#define LGX_DTYPE_BF16 1 /* bf16 storage, fp32 accumulate */

/* layer epilogue modes of lgx_propagate_layer (model.py:163-175: embs.append + stack + mean) */
#define LGX_LAYER_PLAIN 0 /* Y = A X                                                     */
#define LGX_LAYER_FIRST 1 /* Y = A X ; acc = E0 + Y                                      */
#define LGX_LAYER_MID 2   /* Y = A X ; acc += Y                                          */
#define LGX_LAYER_LAST 3  /* out = (acc + A X) / n_mean          (Y not written)         */
#define LGX_LAYER_ONLY 4  /* out = (E0 + A X) / n_mean           (K == 1, Y not written) */
#define LGX_LAYER_PARTIAL 5 /* out = A X in fp32, nothing else (a rank's partial sums of a
                               row-sharded push, reduced across ranks before the epilogue)   */
#define LGX_LAYER_STACK 6 /* out = (E0 + prev[0] + .. + prev[n-1] + A X) / n_mean, the last layer
                             over the kept layer tables (lgx_propagate_layer_stack only)      */

/*
 * A row-partitioned CSR operator plus its launch plan.
 *   indptr [n_rows+1] int64, indices [nnz] int32 (column ids into the X table), vals [nnz] f32.
 *   The plan cuts every row into segments of at most seg_len nonzeros, ordered by length
 *   (longest first); a row with more than one segment is a "split" row whose segments write fp32
 *   partial sums to partials[slot] and are reduced, in slot order (deterministic), by a fix-up
 *   pass.  Built host-side by factors_of_serendipity_recommendation_amd.graph.make_plan().
 *     seg_row  [n_segs]  int32   row of the segment
 *     seg_part [n_segs]  int32   segment index inside its row (0 for unsplit rows)
 *     seg_slot [n_segs]  int32   partial slot, or -1 for an unsplit row
 *     split_row[n_split] int32   split rows
 *     split_ptr[n_split+1] int32 slot range of each split row
 *     partials [n_partials * d] f32 scratch (may be NULL when n_split == 0)
 */
/* A segment launch plan (the fields of lgx_csr above, on their own): one per column block. */
typedef struct lgx_plan {
    const int32_t* seg_row;   /* row ids of the operator (global rows) */
    const int32_t* seg_part;
    const int32_t* seg_slot;
    int64_t n_segs;
    int64_t seg_len;
    const int32_t* split_row;
    const int32_t* split_ptr;
    int64_t n_split;
    int64_t n_partials;
    float* partials;
} lgx_plan;

typedef struct lgx_csr {
    const int64_t* indptr;
    const int32_t* indices;
    const float* vals;
    int64_t n_rows;
    int64_t n_cols;
    int64_t nnz;
    const int32_t* seg_row;
    const int32_t* seg_part;
    const int32_t* seg_slot;
    int64_t n_segs;
    int64_t seg_len;
    const int32_t* split_row;
    const int32_t* split_ptr;
    int64_t n_split;
    int64_t n_partials;
    float* partials;
    /*
     * Optional column blocking of rows [cb_row0, n_rows) -- the item rows of the bipartite operator,
     * which gather the (large) user table.  cb_n = 0: none; the plan above covers every row.
     * cb_n > 0: the plan above covers rows [0, cb_row0) only, and the blocked rows run as cb_n
     * launches, block b over the nonzeros [cb_ptr[b R + r], cb_ptr[(b + 1) R + r]) of row
     * cb_row0 + r (R = n_rows - cb_row0; columns ascending, so a block is one range of columns and
     * its gathers stay inside one 1/cb_n slice of the table: 640 MiB at C4 f32, larger than the
     * 256 MiB MALL, but a narrower working set that measured 57.2 -> 53.6 ms per layer), each with its
     * own plan cb_plans[b] (host array; seg_row holds global rows).  Row sums are carried between
     * the block launches in cb_carry [R, d] f32; the last block adds them and runs the epilogue.
     */
    int64_t cb_row0;
    int64_t cb_n;
    const int64_t* cb_ptr;      /* [(cb_n + 1) * R] int64, device */
    const lgx_plan* cb_plans;   /* [cb_n], host */
    float* cb_carry;            /* [R * d] f32, device */
} lgx_csr;

const char* lgx_version(void);
const char* lgx_last_error(void);
/* arch_out receives e.g. "gfx950:sramecc+:xnack-"; cu/xcd counts from hipDeviceProp_t. */
int lgx_device_info(int device, int* cu_count, int* xcd_count, char* arch_out, size_t arch_len);

/* ---------------------------------------------------------------- a2: graph build */
/* Workspace bytes for lgx_build_norm_adj. */
int lgx_build_norm_adj_workspace(int64_t n_edges, int64_t n_users, int64_t n_items, size_t* ws_bytes);
/*
 * D^-1/2 [[0,R],[R^T,0]] D^-1/2 as CSR over N = n_users + n_items rows, columns sorted.
 * dedup = 0: duplicate (u,i) pairs are summed (PyTorch Loader, dataloader.py:288);
 * dedup = 1: duplicates collapse to 1 (TF Data dok matrix, load_data.py:61).
 * indices / vals must hold 2*n_edges entries; the true nnz is indptr[N] (device) -- read it back
 * when needed.  d_r = (float)(1/sqrt((double)deg_r)) (0 for isolated rows), val = (d_r*a)*d_c:
 * bit-exact with the reference's s_pre_adj_mat.npz.
 */
int lgx_build_norm_adj(const int32_t* user_idx, const int32_t* item_idx, int64_t n_edges,
                       int64_t n_users, int64_t n_items, int dedup, int64_t* indptr,
                       int32_t* indices, float* vals, void* ws, size_t ws_bytes,
                       lgx_stream_t stream);
/* indptr [n_rows+1] from the row ids of a row-sorted (coalesced) COO matrix. */
int lgx_csr_from_coo_rows(const int64_t* coo_rows, int64_t nnz, int64_t n_rows, int64_t* indptr,
                          lgx_stream_t stream);

/* ---------------------------------------------------------------- a4/a5: propagation */
/*
 * One LightGCN layer over the rows of A (row r = local output row r).
 *   X  [n_cols, d]  dtype     input table (columns of A index its rows)
 *   Y  [n_rows, d]  dtype     next-layer table (PLAIN / FIRST / MID)
 *   E0 [n_rows, d]  dtype     layer-0 rows (FIRST / ONLY)
 *   acc[n_rows, d]  f32       running layer sum (FIRST / MID / LAST)
 *   out[n_rows, d]  f32       layer mean (LAST / ONLY), divided by n_mean (= K+1)
 * d: multiple of 4 (f32) or 8 (bf16), <= 1024.
 */
int lgx_propagate_layer(const lgx_csr* A, const void* X, void* Y, const void* E0, float* acc,
                        float* out, int64_t d, int dtype, int mode, float n_mean,
                        lgx_stream_t stream);
/*
 * The epilogue of lgx_propagate_layer alone, on precomputed fp32 row sums y [rows, d] (e.g. the
 * cross-rank sum of LGX_LAYER_PARTIAL outputs): the same per-element arithmetic as the fused path
 * for modes PLAIN..ONLY (Y / E0 / acc / out in the layouts of lgx_propagate_layer).
 */
int lgx_layer_epilogue(const float* y, int64_t rows, void* Y, const void* E0, float* acc, float* out,
                       int64_t d, int dtype, int mode, float n_mean, lgx_stream_t stream);
/*
 * Cross-rank sum of LGX_LAYER_PARTIAL outputs after their exchange (the sharded layer's
 * reduce step): dst[i] = src[0 * slab_elems + i] + src[1 * slab_elems + i] + ... + src[(n_slabs-1) *
 * slab_elems + i], added in slab order in fp32, so the result is independent of how the exchange
 * was chunked and of the collective's own reduction order.  slab_elems a multiple of 4, src / dst
 * 16-B aligned, dst may not overlap src.  Replaces the reference's concat of per-fold SpMM
 * outputs (dataloader.py:319-329, model.py:164-168) on the multi-GPU path.
 */
int lgx_sum_slabs(const float* src, int64_t n_slabs, int64_t slab_elems, float* dst, lgx_stream_t stream);
/*
 * Host-only introspection: the name of the SpMM kernel instantiation lgx_propagate_layer launches
 * for (d, dtype, plan seg_len), e.g. "spmm_segments<bf16,16,1,16>".  Lets tests pin the exact
 * kernel a benchmark configuration times.  No device work.
 */
int lgx_spmm_kernel_name(int64_t d, int dtype, int64_t seg_len, char* buf, size_t len);
/*
 * The last layer over kept layer tables: out = (E0 + prev[0] + ... + prev[n_prev-1] + A X) / n_mean,
 * summed in that order in fp32.  fp32 storage: the same bits as the FIRST / MID / LAST chain.
 * bf16 storage: NOT the same bits -- the chain added each layer's unrounded f32 A X to its f32
 * running sum, the stack adds the bf16-rounded layer tables (one extra bf16 rounding per kept
 * layer, |rel| <= 2^-9 each).  Pinned against the float64 oracle at the bf16 tolerance
 * 2e-2 |ref| + 2e-2 rms(ref) (tests/test_gpu_pinned.py, test_gpu_parity.py).
 * prev: host array of n_prev <= 7 device pointers to [n_rows, d] dtype tables (PLAIN outputs).
 * Per layer this moves (n_prev + 1) dtype tables + one f32 table instead of an f32 running sum
 * read and written every layer.
 */
int lgx_propagate_layer_stack(const lgx_csr* A, const void* X, const void* E0, const void* const* prev,
                              int n_prev, float* out, int64_t d, int dtype, float n_mean, lgx_stream_t stream);
/* Y = A X (alias of lgx_propagate_layer with LGX_LAYER_PLAIN). */
int lgx_spmm_csr(const lgx_csr* A, const void* X, void* Y, int64_t d, int dtype, lgx_stream_t stream);
/* Workspace bytes of lgx_propagate: 2 x [N,d] dtype ping-pong tables + [N,d] f32 layer sum. */
int lgx_propagate_workspace(int64_t n_rows, int64_t d, int dtype, size_t* ws_bytes);
/* Whole K-layer propagation (square A, X = E0 table [N,d] dtype) -> out [N,d] f32 layer mean.
 * When the K-1 intermediate tables fit the workspace (bf16: K <= 5, f32: K <= 4) they are kept
 * and the last layer forms the mean (LGX_LAYER_STACK); otherwise the f32 running sum.  The two
 * schedules give identical fp32 results; in bf16 they differ by the rounding noted above. */
int lgx_propagate(const lgx_csr* A, const void* E0, float* out, int64_t d, int K, int dtype,
                  void* ws, size_t ws_bytes, lgx_stream_t stream);

/* ---------------------------------------------------------------- a6-a9: scoring / top-k */
/*
 * scores[b, i] = <Q[user_rows ? user_rows[b] : b], items[i]>  (optionally sigmoid), f32 [B, n_items].
 * n_items < 2^27 (the score stores use 32-bit lane offsets; LGX_ERR_UNSUPPORTED otherwise).
 */
int lgx_score_dense(const void* Q, const int64_t* user_rows, const void* items, int64_t B,
                    int64_t n_items, int64_t d, int dtype, int apply_sigmoid, float* scores,
                    lgx_stream_t stream);
/* Workspace bytes of lgx_score_topk for this shape: the item-split partial lists, plus 24 parked
 * keys per query half in full-sweep launches (candidates the mask's Bloom filter cannot rule out,
 * settled by exact searches once, at the end of the sweep). */
int lgx_score_topk_workspace(int64_t B, int64_t n_items, int k, size_t* ws_bytes);
/*
 * Fused full-catalog scoring + positive mask + top-k; [B, n_items] is never materialised.
 *   mask_indptr [B+1] int64 / mask_indices int32 sorted per row: items excluded for query b
 *   (may be NULL).  Masked items rank after every unmasked item with value mask_value.
 *   Ranking: higher raw score first, ties -> lower item id.  out_val = raw score, or
 *   sigmoid(score) if apply_sigmoid.  minmax_out (NULL = skip) receives {min, max} of ALL raw
 *   scores (before masking) as f32[2].  k in [1, 256]; k <= 32 (bf16, d a multiple of 32) and
 *   k <= 20 (f32, d a multiple of 64; larger k where the LDS budget allows) run the LDS-staged walk.
 *   Full sweeps over >= 262144 items (and no minmax_out) run as several stream-ordered launches
 *   over consecutive item ranges, each seeding the next through the workspace's lists.
 */
int lgx_score_topk(const void* Q, const int64_t* user_rows, const void* items, int64_t B,
                   int64_t n_items, int64_t d, int dtype, const int64_t* mask_indptr,
                   const int32_t* mask_indices, int k, float mask_value, int apply_sigmoid,
                   int32_t* out_idx, float* out_val, float* minmax_out, void* ws,
                   size_t ws_bytes, lgx_stream_t stream);
/*
 * Host-only introspection: the launch plan lgx_score_topk uses for (B, n_items, d, dtype, k) --
 * kernel, user ranges, full-sweep / catalog-split mode -- as text.  No device work.
 */
int lgx_score_topk_plan(int64_t B, int64_t n_items, int64_t d, int dtype, int k, char* buf, size_t len);
/*
 * Global {min, max} of the raw scores <Q[b], items[i]> over ALL (b, i) -> minmax_out f32[2]: the
 * reference's np.max / np.min of the full user x item dot matrix (recommend.py:163-164, :375-377).
 * The LDS scoring walk with nothing but a running min / max per lane (no top-k state); shapes that
 * walk does not cover go through the top-1 launch of lgx_score_topk.  Needs the workspace below.
 */
int lgx_score_minmax_workspace(int64_t B, int64_t n_items, size_t* ws_bytes);
int lgx_score_minmax(const void* Q, const int64_t* user_rows, const void* items, int64_t B, int64_t n_items,
                     int64_t d, int dtype, float* minmax_out, void* ws, size_t ws_bytes, lgx_stream_t stream);
/* Row-wise top-k of a dense f32 matrix (row stride ld), ties -> lower column.  k in [1, 256]. */
int lgx_topk_rows(const float* S, int64_t rows, int64_t cols, int64_t ld, int k, int32_t* out_idx,
                  float* out_val, lgx_stream_t stream);

/* ---------------------------------------------------------------- a10: metric curves */
/*
 * evaluate_foldout: rankings [users, k] int32 + ragged truths (truth_indptr [users+1] int64,
 * truth_indices int32) -> results [users, 5k] f32 = [precision | recall | ap | ndcg | mrr].
 * inv_log2 [k] f64 = 1/log2(i+2) (host libm values, copied to device by the caller).
 */
int lgx_foldout_metrics(const int32_t* rankings, int64_t users, int k, const int64_t* truth_indptr,
                        const int32_t* truth_indices, const double* inv_log2, float* results,
                        lgx_stream_t stream);
/*
 * batch_test's users' mean of the fold-out curves (LightGCN-tf/utility/batch_test.py:75-76,
 * np.mean(all_result, axis=0) over a float32 [rows, cols] array): out[j] = the float32 sum of
 * src[0][j], src[1][j], ... in row order, divided once in float32 by rows -- numpy's result bit for bit
 * (its axis-0 reduction adds whole rows, it does not block pairwise).  src C-contiguous, rows < 2^24;
 * rows = 0 gives NaN as np.mean of an empty axis does.
 */
int lgx_column_mean_f32(const float* src, int64_t rows, int64_t cols, float* out, lgx_stream_t stream);
/*
 * Procedure.Test's metric sums (lightGCN/LightGCN-PyTorch-master/code/Procedure.py:60-72 over
 * code/utils.py:218-285: getLabel, RecallPrecision_ATk, NDCGatK_r) for all test users at once:
 * rankings [users, k] int32 (k = max topks), test lists as a CSR with each list sorted ascending
 * (truth_indptr [users+1] int64, truth_indices int32, sorted and deduplicated), test_len [users] int64
 * = len(test list) with duplicates (nullable: the CSR lengths), topks [n_topks] int32 ascending in [1, k]
 * (n_topks <= 8), inv_log2 [k] f64 = 1/log2(j+2) -> sums [n_topks, 3] f64, row t = the sums over users
 * for topks[t] of right/|test| (recall), right (precision: divide by the topk) and dcg/idcg (ndcg, idcg
 * over min(topk, |test|) ranks, idcg == 0 -> 1, NaN -> 0): sums[3*t + 0 / 1 / 2].  Summed in a fixed
 * order; workspace from lgx_test_metrics_workspace.
 * Caller contract: topks lives on the device, so the library cannot check it without a host
 * synchronisation: it must be ascending with every entry in [1, k]; an entry outside that range sums
 * to zero.  More than 8 topks: call once per group of 8 (factors_of_serendipity_recommendation_amd/
 * ops.py test_metrics does).
 */
int lgx_test_metrics_workspace(int64_t users, int n_topks, size_t* bytes);
int lgx_test_metrics(const int32_t* rankings, int64_t users, int k, const int64_t* truth_indptr,
                     const int32_t* truth_indices, const int64_t* test_len, const int32_t* topks, int n_topks,
                     const double* inv_log2,
                     double* sums, void* ws, size_t ws_bytes, lgx_stream_t stream);

/* ---------------------------------------------------------------- a11/a12: candidate similarity */
/*
 * scores[p] = <emb_user[row of p], emb_item[cand_items[p]]> for the ragged candidate lists
 * cand_indptr [n_users+1] int64 / cand_items int32 (f32 tables); n_pairs = cand_indptr[n_users]
 * (host value).  n_users = number of candidate lists: emb_user must hold at least that many rows.
 * n_items = rows of emb_item; a candidate id outside [0, n_items) is never read and scores NaN
 * (the Python layer raises IndexError before the launch, as numpy indexing would).
 */
int lgx_gather_scores(const float* emb_user, const float* emb_item, int64_t n_users, int64_t n_items,
                      int64_t d, const int64_t* cand_indptr, const int32_t* cand_items, int64_t n_pairs,
                      float* scores, lgx_stream_t stream);

/* ---------------------------------------------------------------- 8(f) rank 4: stratified candidates */
/*
 * recommend.create_candidates_stratification (recommend.py:359-452):
 * lgx_strat_labels: scores [U, I] f32 (E_user . E_item^T rows) -> labels [U, I] int8 =
 *   floor((f16(s) - min16) / inter16) in numpy's float16 arithmetic, -1 for the user's masked
 *   (train) items (sorted CSR, optional); hist [U, num_fold + 1] int32 label counts.
 * lgx_strat_select: per user, from every label group rint(K * |group| / |eligible|) items
 *   uniformly at random (K = min(targets[u], eligible, out_stride)), in a seed-fixed random order,
 *   padded / trimmed to targets[u] like sample_list -> out [U, out_stride], out_count [U];
 *   out_stride <= 1024.
 */
int lgx_strat_labels(const float* scores, int64_t n_users, int64_t n_items, float min16, float inter16,
                     int num_fold, const int64_t* mask_indptr, const int32_t* mask_indices, int8_t* labels,
                     int32_t* hist, lgx_stream_t stream);
int lgx_strat_select(const int8_t* labels, int64_t n_users, int64_t n_items, const int32_t* hist, int n_bins,
                     const int32_t* targets, uint64_t seed, int32_t* out, int out_stride, int32_t* out_count,
                     lgx_stream_t stream);
/* the same with flags: LGX_STRAT_EXACT runs the radix select for every row (the fast path's
 * cut-and-rank must pick identical sets; used by the parity tests) */
#define LGX_STRAT_EXACT 1
int lgx_strat_select_ex(const int8_t* labels, int64_t n_users, int64_t n_items, const int32_t* hist, int n_bins,
                        const int32_t* targets, uint64_t seed, int32_t* out, int out_stride, int32_t* out_count,
                        int flags, lgx_stream_t stream);
/*
 * Fused form of lgx_score_dense + lgx_strat_labels (recommend.py:375-381): the user x item dots on
 * the matrix cores, labelled in the MFMA epilogue -- the [U, I] f32 score matrix is never written.
 * Labels and hist are bit-identical to the two-step path (same MFMA accumulation order; the float16
 * label arithmetic is a monotone step function of the f32 score, so it is evaluated as a count of
 * thresholds from lgx_strat_thresholds).  Q [n_users, d] (or the rows user_rows), items [n_items, d],
 * f32 or bf16; d / (8 f32 | 16 bf16) in 5..32 chunks (f32 d 40..256, bf16 d 80..256).
 */
int lgx_strat_labels_fused(const void* Q, const int64_t* user_rows, const void* items, int64_t n_users,
                           int64_t n_items, int64_t d, int dtype, float min16, float inter16, int num_fold,
                           const int64_t* mask_indptr, const int32_t* mask_indices, int8_t* labels,
                           int32_t* hist, lgx_stream_t stream);
/* host only: thr[j-1] = the smallest f32 score whose label is >= j, j = 1..num_fold (num_fold < 32) */
int lgx_strat_thresholds(float min16, float inter16, int num_fold, float* thr);
/* label counts of rows of an int8 label matrix, then the user's masked items relabelled -1 and taken
 * out of the counts (the last step of lgx_strat_labels, for labels written by the fused kernel) */
int lgx_strat_hist(int8_t* labels, int64_t n_users, int64_t n_items, int num_fold, const int64_t* mask_indptr,
                   const int32_t* mask_indices, int32_t* hist, lgx_stream_t stream);
/* only the mask step of lgx_strat_hist: masked items of labelled rows -> -1, taken out of hist
 * (for the counts the fused kernel made itself: up to 17 bins) */
int lgx_strat_mask(int8_t* labels, int64_t n_users, int64_t n_items, int num_fold, const int64_t* mask_indptr,
                   const int32_t* mask_indices, int32_t* hist, lgx_stream_t stream);

/* ---------------------------------------------------------------- 8(f) rank 3: interaction files */
/*
 * "uid item item ..." text (dataloader.py:247-277, load_data.py:27-48) parsed on the device in two
 * passes over the same workspace (lgx_parse_lines_workspace):
 *   count: counts_out[0] = numbers in the text, counts_out[1] = lines holding a number (device int64[2])
 *   fill:  line_user [n_lines], line_ptr [n_lines+1] (CSR of each line's items), items [n_numbers - n_lines],
 *          pair_user [n_numbers - n_lines] (optional: the user of every item, file order).
 * A number is a run of decimal digits (int32, saturating); any other byte separates; '
' ends a line.
 */
int lgx_parse_lines_workspace(int64_t n_bytes, size_t* ws_bytes);
int lgx_parse_lines_count(const uint8_t* text, int64_t n_bytes, void* ws, size_t ws_bytes, int64_t* counts_out,
                          lgx_stream_t stream);
int lgx_parse_lines_fill(const uint8_t* text, int64_t n_bytes, const void* ws, size_t ws_bytes, int64_t n_numbers,
                         int64_t n_lines, int32_t* line_user, int64_t* line_ptr, int32_t* items, int32_t* pair_user,
                         lgx_stream_t stream);

/* ---------------------------------------------------------------- 8(f) rank 2: BPR sampling */
/*
 * BPR rows out [n_rows, 2 + neg_num] int32 = [user, a positive, neg_num non-positive items]
 * (sources/sampling.cpp:27-86).  Positives: CSR pos_indptr [n_users+1] int64 / pos_items int32,
 * each user's list SORTED ascending.  users == NULL: row r belongs to user r / per_user
 * (sample_negative, per_user = train_num / user_num); else to users[r] (sample_negative_ByUser).
 * Counter-based draws from `seed` (deterministic per seed; the reference's libc rand() stream is
 * not reproduced).  A user without positives, or an out-of-range user id, gives -1 in its columns
 * 1..; a negative that 4096 draws could not find is -1.
 */
int lgx_sample_bpr(const int64_t* pos_indptr, const int32_t* pos_items, int64_t n_users, int64_t n_items,
                   const int32_t* users, int64_t n_rows, int64_t per_user, int neg_num, uint64_t seed,
                   int32_t* out, lgx_stream_t stream);

/*
 * BPR minibatch loss (model.py:196-209) fused.  light [n_users + n_items, d] f32 = the propagated
 * table (users first); ego_user [n_users, d] / ego_item [n_items, d] f32 = the embedding weights;
 * users / pos / neg int64 [B].  forward writes *out_loss = mean softplus(<u,n> - <u,p>),
 * *out_reg = 0.5 (|U0|^2 + |P0|^2 + |N0|^2) / B, and coef[b] = sigmoid(<u,n> - <u,p>) for backward.
 * An out-of-range index makes the loss NaN.  backward ADDS into g_light / g_user / g_item (dense,
 * caller-zeroed) the gradients of (*grad_loss) * loss + (*grad_reg) * reg (scalars on the device).
 */
int lgx_bpr_loss_workspace(int64_t B, size_t* ws_bytes);
int lgx_bpr_loss_forward(const float* light, const float* ego_user, const float* ego_item, int64_t n_users,
                         int64_t n_items, int64_t d, const int64_t* users, const int64_t* pos, const int64_t* neg,
                         int64_t B, float* coef, float* out_loss, float* out_reg, void* ws, size_t ws_bytes,
                         lgx_stream_t stream);
int lgx_bpr_loss_backward(const float* light, const float* ego_user, const float* ego_item, int64_t n_users,
                          int64_t n_items, int64_t d, const int64_t* users, const int64_t* pos, const int64_t* neg,
                          int64_t B, const float* coef, const float* grad_loss, const float* grad_reg, float* g_light,
                          float* g_user, float* g_item, lgx_stream_t stream);

/*
 * One torch.optim.Adam step (code/utils.py:41: no weight decay, no amsgrad) over n f32 elements in
 * one pass: exp_avg / exp_avg_sq updated in place, param -= lr/(1-beta1^step) * m / (sqrt(v)/sqrt(1-beta2^step) + eps).
 * All four arrays 16-byte aligned; step >= 1 is the step count after this update.
 */
int lgx_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                  double beta1, double beta2, double eps, int64_t step, lgx_stream_t stream);
/* the same with the step count t read from device memory (f32, already advanced for this step), so
 * that a hipGraph-captured training step replays with a live count */
int lgx_adam_step_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                      double beta1, double beta2, double eps, const float* step, lgx_stream_t stream);

/* ---------------------------------------------------------------- 8(f) rank 1: list x list similarity */
#define LGX_REDUCE_MAX 0
#define LGX_REDUCE_SUM 1
/*
 * For every user u (ragged lists A and B as CSR: indptr [U+1] int64, items int32 rows of `table`):
 *   out[p] = max (or sum) over b in B(u) of <table[a_items[p]], table[b]>,  p in [a_indptr[u], a_indptr[u+1]).
 * An empty B(u) gives -inf (max) / 0 (sum).  table [rows, d] f32 or bf16 (fp32 accumulation).
 * Replaces the per-user numpy products of recommend.difference (recommend.py:305-307),
 * utils.ser1_sub (utils.py:34-35), utils.ser2_sub (utils.py:117-121), utils.diversity_sub
 * (utils.py:265-267).
 */
int lgx_list_dot_reduce(const void* table, int64_t d, int dtype, int64_t n_users, const int64_t* a_indptr,
                        const int32_t* a_items, const int64_t* b_indptr, const int32_t* b_items, int reduce,
                        float* out, lgx_stream_t stream);

/* ---------------------------------------------------------------- synthetic graphs (bench) */
/*
 * Deterministic synthetic bipartite edges: user u owns edges [user_offsets[u], user_offsets[u+1]);
 * each edge draws an item by inverse-CDF sampling of item_cdf [n_items] (non-decreasing, last = 1)
 * from a counter-based hash of (seed, edge id), then maps it through item_perm [n_items] (NULL =
 * identity).  n_edges = user_offsets[n_users] (host value).  Same output on every device / rank.
 */
int lgx_synth_edges(uint64_t seed, const int64_t* user_offsets, int64_t n_users,
                    const float* item_cdf, const int32_t* item_perm, int64_t n_items,
                    int64_t n_edges, int32_t* users_out, int32_t* items_out, lgx_stream_t stream);
/* Deterministic N(0, std^2) fill (Box-Muller over a counter hash), dtype f32 or bf16. */
int lgx_fill_normal(void* out, int64_t n, float std, uint64_t seed, int dtype, lgx_stream_t stream);
/* Elements [first, first + n) of the same sequence into out[0, n): a rank fills only its own rows of a
 * table that lgx_fill_normal would fill whole (multi-GPU bench: no replicated [N, d] table). */
int lgx_fill_normal_at(void* out, int64_t first, int64_t n, float std, uint64_t seed, int dtype,
                       lgx_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* LGX_H */
