/*
 * lgx_oracle.c -- CPU restatement of the reference LightGCN propagation / scoring / top-K /
 * fold-out metrics path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product path (liblgx.so, the HIP kernels) never
 * links or calls it.
 *
 * Pinned against reference-produced artefacts (loaded as data, never executed):
 *   - LightGCN-tf/Data/mlls/s_pre_adj_mat.npz : orc_build_norm_adj reproduces indptr/indices/data
 *     bit-exactly from Data/mlls/train.txt;
 *   - LightGCN-tf/weights/mlls/.../emb_{user,item}.npy + output/mlls/LightGCN.result:8 :
 *     orc_propagate(K=4) -> orc_score_topk(-inf mask) -> orc_evaluate_foldout reproduces
 *     recall/precision/ndcg@20 = 0.16075/0.10197/0.14813.
 * Every function cites the reference lines it restates (paths relative to the reference root).
 *
 * Arithmetic conventions (chosen to be the "truth" the fp32 device path is checked against):
 *   - adjacency values: d = (float)(1.0/sqrt((double)deg)) (0 for deg 0), v = (d_r * a) * d_c in
 *     float32 -- equal bit-for-bit to the shipped s_pre_adj_mat.npz;
 *   - propagation / scores: float64 accumulation of float32 inputs.
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return (x > y) - (x < y);
}

/*
 * Normalized bipartite adjacency  A^ = D^-1/2 [[0,R],[R^T,0]] D^-1/2  in CSR.
 *   PyTorch Loader: R = csr_matrix((ones,(u,i))) sums duplicate (u,i) pairs (dataloader.py:288-289),
 *   then lil placement of R / R^T (dataloader.py:349-354), rowsum (:357), np.power(rowsum,-0.5)
 *   with inf->0 (:358-359), D.A.D (:362-363), tocsr (:364).
 *   TF Data: R is a dok matrix assigned R[u,i]=1, i.e. duplicates collapse to 1 (load_data.py:61),
 *   pre_adj built the same way (load_data.py:91-104).
 * dedup=1 selects the TF semantics, dedup=0 the PyTorch semantics.
 * indptr_out [N+1], indices_out/vals_out sized >= 2E.  Returns nnz (or -1 on bad input).
 */
int64_t orc_build_norm_adj(const int32_t* users, const int32_t* items, int64_t n_edges,
                           int64_t n_users, int64_t n_items, int dedup,
                           int64_t* indptr_out, int32_t* indices_out, float* vals_out) {
    const int64_t N = n_users + n_items;
    const int64_t M = 2 * n_edges;
    uint64_t* keys = (uint64_t*)malloc((size_t)(M > 0 ? M : 1) * sizeof(uint64_t));
    float* cnt = (float*)malloc((size_t)(M > 0 ? M : 1) * sizeof(float));
    double* deg = (double*)calloc((size_t)(N > 0 ? N : 1), sizeof(double));
    float* dinv = (float*)malloc((size_t)(N > 0 ? N : 1) * sizeof(float));
    if (!keys || !cnt || !deg || !dinv) return -1;
    for (int64_t e = 0; e < n_edges; ++e) {
        int64_t u = users[e], i = items[e];
        if (u < 0 || u >= n_users || i < 0 || i >= n_items) { free(keys); free(cnt); free(deg); free(dinv); return -1; }
        keys[2 * e] = ((uint64_t)u << 32) | (uint64_t)(n_users + i);
        keys[2 * e + 1] = ((uint64_t)(n_users + i) << 32) | (uint64_t)u;
    }
    qsort(keys, (size_t)M, sizeof(uint64_t), cmp_u64);
    int64_t nnz = 0;
    for (int64_t j = 0; j < M; ++j) {
        if (j == 0 || keys[j] != keys[j - 1]) {
            keys[nnz] = keys[j];
            cnt[nnz] = 1.0f;
            ++nnz;
        } else if (!dedup) {
            cnt[nnz - 1] += 1.0f;  /* csr_matrix sums duplicates (dataloader.py:288) */
        }
    }
    int64_t r = 0;
    indptr_out[0] = 0;
    for (int64_t p = 0; p < nnz; ++p) {
        int64_t row = (int64_t)(keys[p] >> 32);
        while (r < row) indptr_out[++r] = p;
        deg[row] += cnt[p];  /* rowsum (dataloader.py:357) -- exact small integers */
    }
    while (r < N) indptr_out[++r] = nnz;
    for (int64_t v = 0; v < N; ++v)  /* d^-1/2, inf -> 0 (dataloader.py:358-359) */
        dinv[v] = deg[v] > 0 ? (float)(1.0 / sqrt(deg[v])) : 0.0f;
    for (int64_t p = 0; p < nnz; ++p) {
        int64_t row = (int64_t)(keys[p] >> 32);
        int64_t col = (int64_t)(keys[p] & 0xffffffffu);
        indices_out[p] = (int32_t)col;
        volatile float t = dinv[row] * cnt[p];  /* d_mat.dot(adj) (:362) */
        vals_out[p] = t * dinv[col];            /* .dot(d_mat)     (:363) */
    }
    free(keys); free(cnt); free(deg); free(dinv);
    return nnz;
}

/* Y = A^ X for a CSR operator, float64 (model.py:171 torch.sparse.mm(G, all_emb)). */
void orc_spmm_f64(const int64_t* indptr, const int32_t* indices, const float* vals,
                  const double* X, double* Y, int64_t n_rows, int64_t d) {
    for (int64_t r = 0; r < n_rows; ++r) {
        double* y = Y + r * d;
        for (int64_t c = 0; c < d; ++c) y[c] = 0.0;
        for (int64_t p = indptr[r]; p < indptr[r + 1]; ++p) {
            const double v = vals[p];
            const double* x = X + (int64_t)indices[p] * d;
            for (int64_t c = 0; c < d; ++c) y[c] += v * x[c];
        }
    }
}

/*
 * LightGCN.computer() (model.py:145-177): E0 = cat(W_u, W_i) (:149-151), K x sparse.mm (:163-172),
 * mean over the K+1 stacked layers (:173-175).  TF _create_lightgcn_embed is the same math with
 * row folds (LightGCN.py:232-253).  out [N,d] float64; scratch must hold 2*N*d doubles.
 */
void orc_propagate(const int64_t* indptr, const int32_t* indices, const float* vals,
                   const float* E0, int64_t N, int64_t d, int K, double* out, double* scratch) {
    double* cur = scratch;
    double* nxt = scratch + N * d;
    for (int64_t j = 0; j < N * d; ++j) { cur[j] = E0[j]; out[j] = E0[j]; }
    for (int k = 0; k < K; ++k) {
        orc_spmm_f64(indptr, indices, vals, cur, nxt, N, d);
        for (int64_t j = 0; j < N * d; ++j) out[j] += nxt[j];
        double* t = cur; cur = nxt; nxt = t;
    }
    for (int64_t j = 0; j < N * d; ++j) out[j] /= (double)(K + 1);
}

/* ranking order used everywhere: higher score first, ties -> lower item index first */
static int better(double s1, int32_t i1, double s2, int32_t i2) {
    return (s1 > s2) || (s1 == s2 && i1 < i2);
}

/* insert (s,i) into a descending top-k list of current length *len (capacity k) */
static void topk_insert(double* ts, int32_t* ti, int* len, int k, double s, int32_t i) {
    if (*len == k && !better(s, i, ts[k - 1], ti[k - 1])) return;
    int pos = (*len < k) ? *len : k - 1;
    while (pos > 0 && better(s, i, ts[pos - 1], ti[pos - 1])) {
        ts[pos] = ts[pos - 1];
        ti[pos] = ti[pos - 1];
        --pos;
    }
    ts[pos] = s;
    ti[pos] = i;
    if (*len < k) ++*len;
}

/*
 * Row-wise top-k of a dense float32 score matrix: tools.h:13-33 c_top_k_index /
 * c_top_k_array_index (partial_sort_copy by descending rating; the reference leaves tie order
 * unspecified -- this oracle breaks ties by lower index).  out_idx [rows,k] int32.
 * Requires k <= cols.
 */
void orc_topk_rows(const float* S, int64_t rows, int64_t cols, int64_t ld, int k,
                   int32_t* out_idx, float* out_val) {
    double* ts = (double*)malloc(sizeof(double) * (size_t)k);
    int32_t* ti = (int32_t*)malloc(sizeof(int32_t) * (size_t)k);
    for (int64_t r = 0; r < rows; ++r) {
        int len = 0;
        const float* s = S + r * ld;
        for (int64_t c = 0; c < cols; ++c) topk_insert(ts, ti, &len, k, (double)s[c], (int32_t)c);
        for (int j = 0; j < k; ++j) {
            out_idx[r * k + j] = j < len ? ti[j] : -1;
            if (out_val) out_val[r * k + j] = j < len ? (float)ts[j] : -INFINITY;
        }
    }
    free(ts); free(ti);
}

static int in_sorted(const int32_t* a, int64_t n, int32_t x) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo < n && a[lo] == x;
}

/*
 * Full-catalog scoring + positive mask + top-k, never materialising [B,I]:
 *   PyTorch: rating = sigmoid(E_u[users] . E_i^T) (model.py:179-184); rating[u, pos] = -(1<<10)
 *   (Procedure.py:129-134); torch.topk(k) (:135).
 *   TF: batch_ratings = E_u[users] . E_i^T (LightGCN.py:148); rate[u, train] = -inf
 *   (batch_test.py:63-65); c_top_k_index (tools.h:13-22).
 * Q [B,d] (already gathered user rows), items [I,d]; mask CSR over the B query rows with sorted
 * item ids (may be NULL).  Ranking is on the raw dot product (sigmoid is monotone); masked items
 * keep score `mask_value` and therefore rank after every unmasked item.  out_val gets the raw
 * score, or sigmoid(score) when apply_sigmoid (masked entries always get mask_value).
 * minmax (may be NULL) receives the global min / max raw score over ALL B x I pairs
 * (recommend.py:375-377 / :163-164, before masking).
 */
void orc_score_topk(const float* Q, const float* items, int64_t B, int64_t n_items, int64_t d,
                    const int64_t* mask_indptr, const int32_t* mask_indices, int k,
                    float mask_value, int apply_sigmoid, int32_t* out_idx, float* out_val,
                    double* minmax) {
    double* ts = (double*)malloc(sizeof(double) * (size_t)k);
    int32_t* ti = (int32_t*)malloc(sizeof(int32_t) * (size_t)k);
    double mn = INFINITY, mx = -INFINITY;
    for (int64_t b = 0; b < B; ++b) {
        int len = 0;
        const float* q = Q + b * d;
        const int32_t* mrow = mask_indptr ? mask_indices + mask_indptr[b] : NULL;
        int64_t mlen = mask_indptr ? mask_indptr[b + 1] - mask_indptr[b] : 0;
        for (int64_t i = 0; i < n_items; ++i) {
            const float* it = items + i * d;
            double s = 0.0;
            for (int64_t c = 0; c < d; ++c) s += (double)q[c] * (double)it[c];
            if (s < mn) mn = s;
            if (s > mx) mx = s;
            if (mlen && in_sorted(mrow, mlen, (int32_t)i)) continue;
            topk_insert(ts, ti, &len, k, s, (int32_t)i);
        }
        /* fewer than k unmasked items: masked items (all at mask_value) fill the tail in index order */
        for (int64_t j = 0; len < k && j < mlen; ++j) {
            ts[len] = mask_value;
            ti[len] = mrow[j];
            ++len;
        }
        for (int j = 0; j < k; ++j) {
            /* slots past the catalog: index -1, value mask_value */
            int32_t idx = j < len ? ti[j] : -1;
            double s = j < len ? ts[j] : (double)mask_value;
            int masked = (j >= len) || (mlen && in_sorted(mrow, mlen, idx));
            out_idx[b * k + j] = idx;
            if (out_val) {
                if (masked) out_val[b * k + j] = mask_value;
                else out_val[b * k + j] = apply_sigmoid ? (float)(1.0 / (1.0 + exp(-s))) : (float)s;
            }
        }
    }
    if (minmax) { minmax[0] = mn; minmax[1] = mx; }
    free(ts); free(ti);
}

static int in_set(const int32_t* truth, int n, int32_t x) {
    for (int j = 0; j < n; ++j) if (truth[j] == x) return 1;
    return 0;
}

/*
 * evaluate_foldout (evaluate_foldout.h:115-195) with the per-user metric curves
 * precision (:16-30), recall (:32-46), ap (:48-66), ndcg (:68-87), mrr (:89-112).
 * Output row-major [users, 5*top_k] with blocks [pre | rec | ap | ndcg | mrr] (:138-194,
 * apt_evaluate_foldout.pyx:56).  The float/double mix of the C++ source is reproduced: the
 * accumulators are float, each increment is computed in double and added in double precision
 * before being stored back to float.  inv_log2[i] = 1.0/log2(i+2) is passed in (host libm).
 */
void orc_evaluate_foldout(int users_num, const int32_t* rankings, int rank_len,
                          const int64_t* truth_indptr, const int32_t* truth_indices,
                          const double* inv_log2, float* results) {
    for (int u = 0; u < users_num; ++u) {
        const int32_t* rank = rankings + (int64_t)u * rank_len;
        const int32_t* truth = truth_indices + truth_indptr[u];
        const int tl = (int)(truth_indptr[u + 1] - truth_indptr[u]);
        float* out = results + (int64_t)u * 5 * rank_len;
        int hits = 0;
        float sum_pre = 0.0f, dcg = 0.0f, idcg = 0.0f;
        int found = 0;
        for (int i = 0; i < rank_len; ++i) {
            const int hit = in_set(truth, tl, rank[i]);
            if (hit) {
                hits += 1;
                float pre = (float)(1.0 * hits / (i + 1));
                sum_pre += pre;
                dcg = (float)((double)dcg + inv_log2[i]);
            }
            if (i < tl) idcg = (float)((double)idcg + inv_log2[i]);
            out[0 * rank_len + i] = (float)(1.0 * hits / (i + 1));
            out[1 * rank_len + i] = (float)(1.0 * hits / tl);
            out[2 * rank_len + i] = sum_pre / (float)tl;
            out[3 * rank_len + i] = dcg / idcg;
            if (!found && hit) {
                found = 1;
                float rr = (float)(1.0 / (i + 1));
                for (int j = i; j < rank_len; ++j) out[4 * rank_len + j] = rr;
            } else if (!found) {
                out[4 * rank_len + i] = 0.0f;
            }
        }
    }
}
