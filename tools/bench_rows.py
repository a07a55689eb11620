"""Per-row measurement of the SURVEY §8 rows that bench.py does not time (a2, a6, a9, a10, a12 and
the §8(f) rows), each on MI355X against the roofline that bounds it, with the reference's CPU
procedure timed beside it on a bounded sample.  Development / reporting tool, run on the GPU box:

  python tools/bench_rows.py [--out gpurun_out/rows.json] [--only a2,a6]

One JSON object per row.  GPU times are the median of --reps launches bracketed by HIP events on
the stream the ops run on (torch's current stream); inputs are resident in HBM before timing.
Algorithmic bytes / flops per row are stated next to each row in DESIGN.md §5.
The CPU legs use oracle/ (test infrastructure) or the library calls the reference itself makes
(torch / numpy); ``cores`` is the thread count they ran with.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import _lib, ops, recommend, sampling  # noqa: E402
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_edges  # noqa: E402
from oracle import oracle  # noqa: E402  (CPU legs only)

HBM_PEAK = 8.0e12
BF16_PEAK = 2.5e15
F32_PEAK = 157.3e12
DEV = "cuda"
CPU_THREADS = 16


def gpu_ms(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def cpu_s(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


def emit(rows, row, gpu_ms_, units, unit, bound, algo, cpu_units, cpu_seconds, cpu_sample, cpu_cores, note=""):
    """algo: algorithmic bytes (bound hbm) or flops (bound mfma/mfma_f32) per launch"""
    t = gpu_ms_ / 1e3
    peak = {"hbm": HBM_PEAK, "mfma": BF16_PEAK, "mfma_f32": F32_PEAK}[bound]
    r = {"row": row, "gpu_ms": gpu_ms_, "value": units / t, "unit": unit,
         "roofline": {"bound": "hbm" if bound == "hbm" else "mfma",
                      "dtype": {"hbm": None, "mfma": "bf16", "mfma_f32": "f32"}[bound],
                      "achieved": algo / t / (1e9 if bound == "hbm" else 1e12),
                      "peak": peak / (1e9 if bound == "hbm" else 1e12),
                      "unit": "GB/s" if bound == "hbm" else "TFLOP/s", "frac": algo / t / peak,
                      "algorithmic_per_launch": algo},
         "cpu_baseline": {"value": cpu_units / cpu_seconds if cpu_seconds else None, "unit": unit,
                          "cores": cpu_cores, "sample": cpu_sample, "seconds": cpu_seconds},
         "note": note}
    r["speedup_vs_cpu"] = r["value"] / r["cpu_baseline"]["value"] if r["cpu_baseline"]["value"] else None
    print(json.dumps(r), flush=True)
    rows.append(r)


# ---------------------------------------------------------------------------------------------- a2
def row_a2(rows, reps):
    """lgx_build_norm_adj at C4 (500 M edges -> 1e9 nnz), plan excluded (dataloader.py:339-376)."""
    cfg = CONFIGS["synth10m"]
    u, i = synth_edges(cfg, 2020, DEV)
    E, U, I = int(u.numel()), cfg.n_users, cfg.n_items
    N = U + I
    L = _lib.lib()
    ws = ctypes.c_size_t(0)
    _lib.check(L.lgx_build_norm_adj_workspace(E, U, I, ctypes.byref(ws)), "ws")
    indptr = torch.empty(N + 1, dtype=torch.int64, device=DEV)
    indices = torch.empty(2 * E, dtype=torch.int32, device=DEV)
    vals = torch.empty(2 * E, dtype=torch.float32, device=DEV)
    work = torch.empty(ws.value, dtype=torch.uint8, device=DEV)
    st = torch.cuda.current_stream().cuda_stream

    def run():
        _lib.check(L.lgx_build_norm_adj(u.data_ptr(), i.data_ptr(), E, U, I, 1, indptr.data_ptr(),
                                        indices.data_ptr(), vals.data_ptr(), work.data_ptr(), ws.value, st),
                   "lgx_build_norm_adj")
    ms = gpu_ms(run, max(1, reps // 2))
    algo = E * 8 + 2 * E * 8 + (N + 1) * 8  # read the pairs, write indices + values, indptr
    del indices, vals, work, indptr
    # CPU: the oracle's restatement of the scipy build (C, one thread) on the ML-1M-shaped graph
    c1 = CONFIGS["ml1m"]
    cu, ci = synth_edges(c1, 2020, DEV)
    cu, ci = cu.cpu().numpy(), ci.cpu().numpy()
    s = cpu_s(lambda: oracle.build_norm_adj(cu, ci, c1.n_users, c1.n_items, dedup=True))
    emit(rows, "a2 adjacency build (lgx_build_norm_adj)", ms, E, "edges/s", "hbm", algo, len(cu), s,
         f"ML-1M-shaped graph ({len(cu)} edges), oracle C restatement", 1,
         "radix sort of packed keys + 5 streaming passes; algorithmic = 8 B/edge in + 16 B/nnz out")
    del u, i
    torch.cuda.empty_cache()


# ------------------------------------------------------------------------------------- a6 + a9
def row_a6_a9(rows, reps):
    """getUsersRating [B, I] = sigmoid(E_u[users] E_i^T) (model.py:179-184) and the row top-K of
    tools.h:13-33 on it: bf16 [4096, 1M] d=256 (SURVEY C5 inputs; write-bound), then the reference's
    fp32 at its own test batch (B=100, parse.py:26) and at [4096, 1M] (both f32-MFMA-bound)."""
    B, I, d, k = 4096, 1_000_000, 256, 20
    Q = ops.fill_normal((B, d), 1.0 / 16, 1, dtype=torch.bfloat16)
    items = ops.fill_normal((I, d), 1.0 / 16, 2, dtype=torch.bfloat16)
    S = ops.score_dense(Q, items, apply_sigmoid=True)
    ms = gpu_ms(lambda: ops.score_dense(Q, items, apply_sigmoid=True), reps)
    ms_raw = gpu_ms(lambda: ops.score_dense(Q, items), reps)
    Qc, Ic = Q[:64].float().cpu(), items.float().cpu()
    torch.set_num_threads(CPU_THREADS)
    s = cpu_s(lambda: torch.sigmoid(torch.matmul(Qc, Ic.t())))
    emit(rows, "a6 dense scoring, bf16 (lgx_score_dense, sigmoid)", ms, B * I, "scores/s", "hbm",
         4 * B * I + 2 * I * d + 2 * B * d, 64 * I, s, f"64 users x {I} items, d={d} fp32 torch.matmul + sigmoid",
         CPU_THREADS, f"bf16 in, f32 out [B, I]; flops {2 * B * I * d:.3g} (MFMA well under its roof: write-bound); "
                      f"raw scores (TF batch_ratings, no sigmoid) {ms_raw:.2f} ms")
    ms = gpu_ms(lambda: ops.topk_rows(S, k), reps)
    Sc = S[:256].cpu()
    s = cpu_s(lambda: torch.topk(Sc, k))
    emit(rows, "a9 row top-K (lgx_topk_rows)", ms, B * I, "scores/s", "hbm", 4 * B * I + 8 * B * k,
         256 * I, s, f"256 rows x {I} torch.topk(k={k})", CPU_THREADS)
    del S, Q, items
    torch.cuda.empty_cache()
    # the reference's precision: fp32 tables, fp32 products (model.py:183)
    items = ops.fill_normal((I, d), 1.0 / 16, 2)
    Ic = items.cpu()
    for Bf in (100, 4096):
        Q = ops.fill_normal((Bf, d), 1.0 / 16, 3)
        ms = gpu_ms(lambda: ops.score_dense(Q, items, apply_sigmoid=True), reps)
        nc = min(Bf, 64)
        Qc = Q[:nc].cpu()
        s = cpu_s(lambda: torch.sigmoid(torch.matmul(Qc, Ic.t())))
        emit(rows, f"a6 dense scoring, fp32 B={Bf} (lgx_score_dense, sigmoid)", ms, Bf * I, "scores/s", "mfma_f32",
             2.0 * Bf * I * d, nc * I, s, f"{nc} users x {I} items, d={d} fp32 torch.matmul + sigmoid", CPU_THREADS,
             f"f32 in, f32 out [{Bf}, {I}] ({4 * Bf * I / 1e9:.2f} GB written: "
             f"{4 * Bf * I / HBM_PEAK * 1e3:.3f} ms at the HBM peak) -- bound by the f32 MFMA flops")
        del Q
    del items
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------------------------- a10
def row_a10(rows, reps):
    """evaluate_foldout (evaluate_foldout.h:115-195) for 1 M users, top-20, 10 truths each."""
    users, k, T, I = 1_000_000, 20, 10, 1_000_000
    g = torch.Generator(device=DEV).manual_seed(5)
    rank = torch.randint(0, I, (users, k), device=DEV, dtype=torch.int32, generator=g)
    tp = torch.arange(0, users * T + 1, T, device=DEV, dtype=torch.int64)
    ti = torch.randint(0, I, (users * T,), device=DEV, dtype=torch.int32, generator=g)
    ms = gpu_ms(lambda: ops.foldout_metrics(rank, (tp, ti)), reps)
    n = 100_000
    r_h = rank[:n].cpu().numpy()
    t_h = ti[:n * T].cpu().numpy().reshape(n, T).tolist()
    s = cpu_s(lambda: oracle.evaluate_foldout(r_h, t_h))
    emit(rows, "a10 fold-out metrics (lgx_foldout_metrics)", ms, users, "users/s", "hbm",
         users * (4 * k + 4 * T + 8 + 4 * 5 * k), n, s, f"{n} users, oracle C restatement", 1)


# ---------------------------------------------------------------------------------------------- a12
def row_a12(rows, reps):
    """recommend.accuracy_cf (recommend.py:208-223): 1000 candidates per user, d=64 fp32, top-20."""
    U, I, C, d, K = 100_000, 1_000_000, 1000, 64, 20
    eu = ops.fill_normal((U, d), 0.1, 3)
    ei = ops.fill_normal((I, d), 0.1, 4)
    g = torch.Generator(device=DEV).manual_seed(6)
    cand = torch.randint(0, I, (U * C,), device=DEV, dtype=torch.int32, generator=g)
    cp = torch.arange(0, U * C + 1, C, device=DEV, dtype=torch.int64)

    def run():
        sc = ops.gather_scores(eu, ei, (cp, cand), U * C)
        return ops.topk_rows(sc.view(U, C), K)
    ms = gpu_ms(run, reps)
    n = 2000
    eu_h, ei_h = eu[:n].cpu().numpy(), ei.cpu().numpy()
    c_h = cand[:n * C].cpu().numpy().reshape(n, C)

    def cpu():  # the reference's per-user numpy dot + argpartition (recommend.py:214-217, :53-56)
        for u in range(n):
            s_ = np.dot(ei_h[c_h[u]], eu_h[u])
            np.argpartition(s_, -K)[-K:]
    s = cpu_s(cpu)
    emit(rows, "a12 candidate scoring + top-K (lgx_gather_scores + lgx_topk_rows)", ms, U * C, "pairs/s", "hbm",
         U * C * (4 + 4 * d + 4) + U * d * 4 + U * C * 4 + U * K * 8, n * C, s,
         f"{n} users x {C} candidates, numpy dot + argpartition per user", 1,
         "gathered item rows counted at 4*d B each (table 256 MB: L2/MALL serve part of them)")


# ------------------------------------------------------------------------------------------ (f) 1
def row_f1(rows, reps):
    """recommend.difference max-dot of candidates vs train history (recommend.py:287-312)."""
    U, I, C, H, d = 20_000, 1_000_000, 1000, 50, 64
    ei = ops.fill_normal((I, d), 0.1, 7)
    g = torch.Generator(device=DEV).manual_seed(8)
    a = (torch.arange(0, U * C + 1, C, device=DEV, dtype=torch.int64),
         torch.randint(0, I, (U * C,), device=DEV, dtype=torch.int32, generator=g))
    b = (torch.arange(0, U * H + 1, H, device=DEV, dtype=torch.int64),
         torch.randint(0, I, (U * H,), device=DEV, dtype=torch.int32, generator=g))
    ms = gpu_ms(lambda: ops.list_dot_reduce(ei, a, b, "max"), reps)
    n = 300
    T = ei.cpu().numpy()
    A = a[1][:n * C].cpu().numpy().reshape(n, C)
    Bh = b[1][:n * H].cpu().numpy().reshape(n, H)

    def cpu():  # recommend.py:305-307: numpy dot of the candidate and history rows, max per candidate
        for u in range(n):
            (T[A[u]] @ T[Bh[u]].T).max(axis=1)
    s = cpu_s(cpu)
    emit(rows, "f1 list x list max-dot (lgx_list_dot_reduce)", ms, U * C * H, "dots/s", "mfma_f32",
         2.0 * U * C * H * d, n * C * H, s, f"{n} users x {C} x {H}, numpy f32 per user", 1,
         "f32 tables: priced against the 157 TF f32 matrix peak")


# ------------------------------------------------------------------------------------------ (f) 2
def _np_sample(indptr, items, n_items, rng):
    """Vectorised restatement of sampling.cpp:27-86 (one positive + one negative per train row,
    negatives redrawn while they hit the user's positives)."""
    n_users = len(indptr) - 1
    deg = np.diff(indptr)
    users = np.repeat(np.arange(n_users, dtype=np.int64), deg)
    pos = items[indptr[users] + rng.integers(0, deg[users])]
    keys = users * n_items + items.astype(np.int64)  # sorted: CSR rows ascending, items sorted
    neg = rng.integers(0, n_items, len(users))
    todo = np.arange(len(users))
    while len(todo):
        q = users[todo] * n_items + neg[todo]
        j = np.minimum(np.searchsorted(keys, q), len(keys) - 1)
        hit = keys[j] == q
        todo = todo[hit]
        neg[todo] = rng.integers(0, n_items, len(todo))
    return users, pos, neg


def row_f2(rows, reps):
    """UniformSample_original through lgx_sample_bpr: one (user, pos, neg) row per train edge."""
    U, I, P = 1_000_000, 1_000_000, 50
    g = torch.Generator(device=DEV).manual_seed(9)
    it = torch.randint(0, I, (U, P), device=DEV, dtype=torch.int32, generator=g)
    it = torch.sort(it, dim=1).values.reshape(-1).contiguous()
    ip = torch.arange(0, U * P + 1, P, device=DEV, dtype=torch.int64)
    ms = gpu_ms(lambda: sampling.sample_device((ip, it), I, per_user=P, seed_value=1, drop_invalid=False), reps)
    n = 200_000
    ip_h, it_h = ip[:n + 1].cpu().numpy(), it[:n * P].cpu().numpy()
    s = cpu_s(lambda: _np_sample(ip_h, it_h, I, np.random.default_rng(1)))
    emit(rows, "f2 BPR sampler (lgx_sample_bpr)", ms, U * P, "samples/s", "hbm", U * P * (12 + 4 * 6) + U * 8, n * P, s,
         f"{n} users x {P} rows, vectorised numpy restatement", 1,
         "algorithmic: 12 B row out + ~6 probes of 4 B (positive draw + binary search) per row")


def _bpr_step_cpu(G, user_w, item_w, opt, users, pos, neg, K, decay):
    """One minibatch of the reference's BPR step on the host, restated with its own torch calls:
    computer() (model.py:145-177) + bpr_loss (model.py:186-209) + utils.BPRLoss.stageOne (Adam)."""
    all_emb = torch.cat([user_w, item_w])
    embs = [all_emb]
    for _ in range(K):
        all_emb = torch.sparse.mm(G, all_emb)
        embs.append(all_emb)
    out = torch.mean(torch.stack(embs, dim=1), dim=1)
    U = user_w.shape[0]
    ue, pe, ne = out[:U][users], out[U:][pos], out[U:][neg]
    reg = 0.5 * (user_w[users].norm(2).pow(2) + item_w[pos].norm(2).pow(2) + item_w[neg].norm(2).pow(2)) / len(users)
    loss = torch.mean(torch.nn.functional.softplus((ue * ne).sum(1) - (ue * pe).sum(1))) + decay * reg
    opt.zero_grad()
    loss.backward()
    opt.step()


def row_f2b(rows, reps, tmpdir):
    """One BPR training epoch (Procedure.BPR_train_original, Procedure.py:26-57) on the Gowalla-shaped
    graph (BASELINE configs[0]: 29,858 x 40,981, 810,128 edges, K=3, d=64 fp32, batch 2048)."""
    from factors_of_serendipity_recommendation_amd import train as lgx_train
    from factors_of_serendipity_recommendation_amd.dataloader import Loader
    from factors_of_serendipity_recommendation_amd.model import LightGCN
    cfg = CONFIGS["gowalla"]
    u, i = synth_edges(cfg, 2020, DEV)
    u, i = u.cpu().numpy(), i.cpu().numpy()
    path = os.path.join(tmpdir, "rows_gowalla")
    os.makedirs(path, exist_ok=True)
    order = np.argsort(u, kind="stable")
    u, i = u[order], i[order]
    bounds = np.searchsorted(u, np.arange(cfg.n_users + 1))
    with open(os.path.join(path, "train.txt"), "w") as f:
        for x in range(cfg.n_users):
            if bounds[x + 1] > bounds[x]:
                f.write(str(x) + " " + " ".join(map(str, i[bounds[x]:bounds[x + 1]])) + "\n")
    with open(os.path.join(path, "test.txt"), "w") as f:
        f.write(f"0 {int(i[0])}\n")
    ds = Loader(path=path, device=DEV, cache_adj=False)
    conf = {"latent_dim_rec": cfg.d, "lightGCN_n_layers": cfg.K, "keep_prob": 0.6, "A_split": False,
            "pretrain": 0, "dropout": 0, "decay": 1e-4, "lr": 0.001}
    torch.manual_seed(0)
    model = LightGCN(conf, ds).to(DEV)
    bpr = lgx_train.BPRLoss(model, conf)
    lgx_train.BPR_train_original(ds, model, bpr, 0, batch_size=2048, device=DEV)  # warm-up epoch
    ms = gpu_ms(lambda: lgx_train.BPR_train_original(ds, model, bpr, 1, batch_size=2048, device=DEV),
                max(1, reps // 2))
    if os.environ.get("LGX_ROWS_F2B_FUSED_ONLY"):  # profiling: only the product epochs
        print(f"f2b epoch {ms:.1f} ms", flush=True)
        return
    model.bpr_loss = model.bpr_loss_torch  # A/B: the reference's torch-op loss in the same epoch
    ms_torch_loss = gpu_ms(lambda: lgx_train.BPR_train_original(ds, model, bpr, 2, batch_size=2048, device=DEV),
                           max(1, reps // 2))
    del model.bpr_loss
    E = ds.trainDataSize
    n_batches = E // 2048 + 1
    A = model._csr
    nnz, N, d = A.nnz, cfg.n_users + cfg.n_items, cfg.d
    spmm_bytes = nnz * (8 + 4 * d) + N * d * 4 + 8 * (N + 1)
    # CPU: the reference's minibatch on the host (torch.sparse.mm COO, 16 threads), a few batches
    from oracle.torch_ref import coo_from_csr
    torch.set_num_threads(CPU_THREADS)
    G = coo_from_csr(A.indptr.cpu().numpy(), A.indices.cpu().numpy(), A.vals.cpu().numpy(), N)
    uw = torch.nn.Parameter(torch.randn(cfg.n_users, d) * 0.1)
    iw = torch.nn.Parameter(torch.randn(cfg.n_items, d) * 0.1)
    opt = torch.optim.Adam([uw, iw], lr=0.001)
    rng = np.random.default_rng(0)
    nb = 8
    bu = [torch.from_numpy(rng.integers(0, cfg.n_users, 2048)) for _ in range(nb)]
    bp = [torch.from_numpy(rng.integers(0, cfg.n_items, 2048)) for _ in range(nb)]
    bn = [torch.from_numpy(rng.integers(0, cfg.n_items, 2048)) for _ in range(nb)]
    _bpr_step_cpu(G, uw, iw, opt, bu[0], bp[0], bn[0], cfg.K, 1e-4)
    s = cpu_s(lambda: [_bpr_step_cpu(G, uw, iw, opt, bu[j], bp[j], bn[j], cfg.K, 1e-4) for j in range(nb)])
    emit(rows, "f2b BPR training epoch (lgx_sample_bpr + 2K lgx_propagate_layer + lgx_bpr_loss_* + lgx_adam_step per minibatch)", ms, E,
         "train edges/s", "hbm", n_batches * 2 * cfg.K * spmm_bytes, nb * 2048, s,
         f"{nb} minibatches of 2048 on the host: torch.sparse.mm x K + mean + BPR loss + Adam (model.py:145-209), "
         "sampling excluded", CPU_THREADS,
         f"{n_batches} minibatches per epoch; algorithmic = the 2K f32 SpMM layers of every minibatch; "
         f"with the torch-op loss instead of lgx_bpr_loss_*: {ms_torch_loss:.1f} ms")


# ------------------------------------------------------------------------------------------ (f) 3
def row_f3(rows, reps, tmpdir):
    """The uid item item ... train.txt parser (dataloader.py:247-277) on the device."""
    rng = np.random.default_rng(10)
    n_lines, per = 200_000, 50
    its = rng.integers(0, 1_000_000, (n_lines, per))
    lines = [str(u) + " " + " ".join(map(str, its[u])) for u in range(n_lines)]
    data = ("\n".join(lines) + "\n").encode()
    text = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(DEV)
    ms = gpu_ms(lambda: ops.parse_lines(text), reps)
    n = 20_000
    path = os.path.join(tmpdir, "rows_train.txt")
    with open(path, "wb") as f:
        f.write(("\n".join(lines[:n]) + "\n").encode())
    s = cpu_s(lambda: oracle.parse_lightgcn_txt(path, path))
    emit(rows, "f3 interaction-file parse (lgx_parse_lines_count/fill)", ms, len(data), "bytes/s", "hbm",
         len(data) + n_lines * per * 8 + n_lines * 12, len("\n".join(lines[:n]).encode()), s,
         f"{n} lines, python line loop (oracle restatement of the Loader)", 1)


# ------------------------------------------------------------------------------------------ (f) 4
def row_f4(rows, reps):
    """create_candidates_stratification labels + per-label picks (recommend.py:314-452), one
    4096-user batch against 1 M items, d=64 fp32."""
    B, I, d, F, Kc = 4096, 1_000_000, 64, 10, 1000
    eu = ops.fill_normal((B, d), 0.1, 11)
    ei = ops.fill_normal((I, d), 0.1, 12)
    g = torch.Generator(device=DEV).manual_seed(13)
    mi = torch.sort(torch.randint(0, I, (B, 50), device=DEV, dtype=torch.int32, generator=g), dim=1).values
    mi = mi.reshape(-1).contiguous()
    mp = torch.arange(0, B * 50 + 1, 50, device=DEV, dtype=torch.int64)
    min16, inter16 = recommend.stratification_bounds(eu, ei, F, 0.1)
    L = _lib.lib()
    st = torch.cuda.current_stream().cuda_stream
    S = ops.score_dense(eu, ei)
    labels = torch.empty((B, I), dtype=torch.int8, device=DEV)
    hist = torch.empty((B, F + 1), dtype=torch.int32, device=DEV)
    tgt = torch.full((B,), Kc, dtype=torch.int32, device=DEV)
    out = torch.empty((B, Kc), dtype=torch.int32, device=DEV)
    cnt = torch.empty(B, dtype=torch.int32, device=DEV)

    def lab():
        _lib.check(L.lgx_strat_labels(S.data_ptr(), B, I, min16, inter16, F, mp.data_ptr(), mi.data_ptr(),
                                      labels.data_ptr(), hist.data_ptr(), st), "lgx_strat_labels")

    def fused():
        _lib.check(L.lgx_strat_labels_fused(eu.data_ptr(), None, ei.data_ptr(), B, I, d, _lib.LGX_DTYPE_F32, min16,
                                            inter16, F, mp.data_ptr(), mi.data_ptr(), labels.data_ptr(),
                                            hist.data_ptr(), st), "lgx_strat_labels_fused")

    def hist_only():
        _lib.check(L.lgx_strat_hist(labels.data_ptr(), B, I, F, None, None, hist.data_ptr(), st), "lgx_strat_hist")

    def sel():
        _lib.check(L.lgx_strat_select(labels.data_ptr(), B, I, hist.data_ptr(), F + 1, tgt.data_ptr(), 77,
                                      out.data_ptr(), Kc, cnt.data_ptr(), st), "lgx_strat_select")
    def fused20():  # > 16 folds: the labels alone in the MFMA epilogue, the counts by a separate pass
        _lib.check(L.lgx_strat_labels_fused(eu.data_ptr(), None, ei.data_ptr(), B, I, d, _lib.LGX_DTYPE_F32, min16,
                                            inter16, 20, mp.data_ptr(), mi.data_ptr(), labels.data_ptr(),
                                            hist20.data_ptr(), st), "lgx_strat_labels_fused")
    hist20 = torch.empty((B, 21), dtype=torch.int32, device=DEV)
    ms_s = gpu_ms(lambda: ops.score_dense(eu, ei), reps)
    ms_l = gpu_ms(lab, reps)
    ms_f20 = gpu_ms(fused20, reps)
    ms_f = gpu_ms(fused, reps)
    ms_h = gpu_ms(hist_only, reps)
    fused()
    ms_p = gpu_ms(sel, reps)
    n = 200
    eu_h, ei_h = eu[:n].cpu().numpy(), ei.cpu().numpy()
    tr = mi[:n * 50].cpu().numpy().reshape(n, 50).tolist()
    s = cpu_s(lambda: oracle.stratification_labels(eu_h, ei_h, tr, F, 0.1))
    emit(rows, "f4 stratified candidates: fused scores->labels + select (lgx_strat_labels_fused, "
         "lgx_strat_select)", ms_f + ms_p, B * I, "user-item pairs/s", "mfma_f32", 2.0 * B * I * d,
         n * I, s, f"{n} users x {I} items: numpy dot + float16 labels + histograms (labels only)", 1,
         f"per batch: fused labels + counts {ms_f:.2f} ms (the counting pass over the labels it replaces: "
         f"{ms_h:.2f} ms), select "
         f"{ms_p:.2f} ms; 20 folds (labels in the MFMA epilogue, counts by a separate pass) {ms_f20:.2f} ms; "
         f"the two-step path: score_dense {ms_s:.2f} + labels {ms_l:.2f} ms; roofline: the "
         "fused kernel's f32 MFMA flops over the whole batch time")
    del S, labels
    torch.cuda.empty_cache()


# ----------------------------------------------------------------------------------- a7 / a8 e2e
def _eval_dataset(cfg, tmpdir):
    """A synthetic dataset of the config's shape in the reference's txt format: every 5th edge of a
    user (sorted by item) is a test interaction, the rest train (users with < 2 edges: train only)."""
    from factors_of_serendipity_recommendation_amd.dataloader import Loader
    u, i = synth_edges(cfg, 2020, DEV)
    u, i = u.cpu().numpy(), i.cpu().numpy()
    order = np.lexsort((i, u))
    u, i = u[order], i[order]
    bounds = np.searchsorted(u, np.arange(cfg.n_users + 1))
    pos = np.arange(len(u)) - bounds[u]
    deg = np.diff(bounds)[u]
    test = (pos % 5 == 4) & (deg >= 2)
    path = os.path.join(tmpdir, f"rows_eval_{cfg.name}")
    os.makedirs(path, exist_ok=True)
    for name, sel in (("train.txt", ~test), ("test.txt", test)):
        uu, ii = u[sel], i[sel]
        b = np.searchsorted(uu, np.arange(cfg.n_users + 1))
        with open(os.path.join(path, name), "w") as f:
            for x in range(cfg.n_users):
                if b[x + 1] > b[x]:
                    f.write(str(x) + " " + " ".join(map(str, ii[b[x]:b[x + 1]])) + "\n")
    return Loader(path=path, device=DEV, cache_adj=False)


def row_eval(rows, reps, tmpdir, cfg_name):
    """The reference's evaluation loops end to end on a synthetic graph of the config's shape:
    Procedure.Test (Procedure.py:96-174; evaluator.Test: one propagation, one fused score + mask +
    top-20 launch, host metrics) and TF batch_test.test (batch_test.py:25-84; evaluator.batch_test on
    the propagated tables: fused score + -inf mask + top-20 + fold-out curves).  Phases timed apart
    (device synchronised between them) to give the host metric share.  CPU legs: the reference's own
    procedure restated with its library calls on a bounded sample -- Procedure.Test recomputes the
    K-layer propagation for every 100-user batch (model.py:180) -- extrapolated to every test user."""
    from factors_of_serendipity_recommendation_amd import evaluator
    from factors_of_serendipity_recommendation_amd.model import LightGCN
    from oracle import torch_ref
    cfg = CONFIGS[cfg_name]
    ds = _eval_dataset(cfg, tmpdir)
    conf = {"latent_dim_rec": cfg.d, "lightGCN_n_layers": cfg.K, "keep_prob": 0.6, "A_split": False,
            "pretrain": 0, "dropout": 0}
    torch.manual_seed(0)
    model = LightGCN(conf, ds).to(DEV).eval()
    users = list(ds.testDict.keys())
    n_test = len(users)

    def sync_t():
        torch.cuda.synchronize()
        return time.perf_counter()

    def test_once():
        model._eval_cache = None  # propagate again, as a call after a training epoch does
        return evaluator.Test(ds, model, topks=[20])
    res = test_once()
    # evaluator.Test's steps one by one (the device synchronised at each boundary), so that the wall
    # time and its phase split come from the same runs
    # (the first call above built the test lists -- row ids, mask CSR, test-item keys -- once; a later
    # Procedure.Test call over the same testDict reuses them, as these do)
    ph = {"propagation": [], "lists": [], "score_topk": [], "hits_metrics": []}
    walls = []
    for _ in range(reps):
        model._eval_cache = None
        t0 = sync_t()
        with torch.no_grad():
            all_users, all_items = model.computer()
        t1 = sync_t()
        tl = evaluator._TestLists.get(ds, all_items.shape[0], all_users.device)
        t2 = sync_t()
        idx = tl.route(all_items.shape[0], 20, cfg.d).topk(all_users, all_items, 20, -float(1 << 10), True)
        t3 = sync_t()
        ops.test_metrics(idx, tl.truth, [20], tl.recall_n_dev).cpu()  # as evaluator.Test: one launch + the sums' copy
        t4 = sync_t()
        for k_, a_, b_ in (("propagation", t0, t1), ("lists", t1, t2), ("score_topk", t2, t3),
                           ("hits_metrics", t3, t4)):
            ph[k_].append((b_ - a_) * 1e3)
        walls.append(t4 - t0)
    ph = {k_: float(np.median(v)) for k_, v in ph.items()}
    ms = float(np.median(walls)) * 1e3
    # CPU: Procedure.Test's per-batch body on the host (computer() + getUsersRating + mask + topk +
    # test_one_batch), 3 batches of 100 users, extrapolated to ceil(n_test / 100) batches
    A = model._csr
    N = cfg.n_users + cfg.n_items
    G = torch_ref.coo_from_csr(A.indptr.cpu().numpy(), A.indices.cpu().numpy(), A.vals.cpu().numpy(), N)
    E0 = torch.cat([model.embedding_user.weight, model.embedding_item.weight]).detach().float().cpu()
    torch.set_num_threads(CPU_THREADS)
    nb = 3
    pos_lists = ds.getUserPosItems(users[:100 * nb])

    def cpu_batches():
        for j in range(nb):
            out = torch_ref.propagate_cpu(G, E0, cfg.K)
            Eu, Ei = out[:cfg.n_users], out[cfg.n_users:]
            bu = users[100 * j:100 * (j + 1)]
            rk, _ = torch_ref.score_topk_cpu(Eu[torch.as_tensor(bu)], Ei, 20, pos_lists[100 * j:100 * (j + 1)])
            oracle.torch_style_metrics(rk.numpy(), [ds.testDict[x] for x in bu], [20])
    s = cpu_s(cpu_batches)
    n_batches = -(-n_test // 100)
    emit(rows, f"a7 Procedure.Test end to end, {cfg.name} shape (evaluator.Test)", ms, n_test, "test users/s", "hbm",
         0, 100 * nb, s,
         f"{nb} of the reference's 100-user batches (K={cfg.K} torch.sparse.mm propagation + matmul + sigmoid + "
         f"mask + torch.topk + per-user metric loops each), extrapolated to {n_batches} batches", CPU_THREADS,
         f"{cfg.n_users} x {cfg.n_items}, {A.nnz} nnz, K={cfg.K}, d={cfg.d} fp32, {n_test} test users; phases (ms): "
         + ", ".join(f"{k_} {v:.2f}" for k_, v in ph.items())
         + f"; host share (lists + hits / metric sums) {(ph['lists'] + ph['hits_metrics']) / sum(ph.values()):.2f}; "
           f"recall@20 {float(res['recall'][0]):.5f} (synthetic graph)")
    # the score + mask + top-20 step inside the loop (the fused launch for most users, the dense route
    # for users with long masks), against the f32 MFMA peak (its own HIP-event timing)
    rt = tl.route(all_items.shape[0], 20, cfg.d)
    ms_k = gpu_ms(lambda: rt.topk(all_users, all_items, 20, -float(1 << 10), True), reps)
    fl = 2.0 * n_test * cfg.n_items * cfg.d
    n_light = n_test - rt.n_heavy
    plan = ops.score_topk_plan(n_light, cfg.n_items, cfg.d, torch.float32, 20)
    rows[-1]["roofline"] = {"bound": "mfma_f32", "kernel": plan + f"; {rt.n_heavy} users with > "
                            f"{rt.thr} masked items by the dense route (score_dense_lds + "
                            "topk_rows_kernel)", "launch_ms": ms_k,
                            "achieved": fl / (ms_k / 1e3) / 1e12, "peak": F32_PEAK / 1e12, "unit": "TFLOP/s",
                            "frac": fl / (ms_k / 1e3) / F32_PEAK,
                            "note": "the score + mask + top-20 step of the loop (every test user); the loop's "
                                    "other phases above"}
    rows[-1]["phases_ms"] = ph
    # TF batch_test on the propagated tables (LightGCN.py:148 ratings, batch_test.py:47-83)
    with torch.no_grad():
        all_users, all_items = model.computer()
    train_items = {x: ds.allPos[x] for x in users}
    test_set = {x: ds.testDict[x] for x in users}
    evaluator.batch_test(all_users, all_items, users, train_items, test_set, Ks=[20])
    bw = []
    for _ in range(reps):
        t0 = sync_t()
        evaluator.batch_test(all_users, all_items, users, train_items, test_set, Ks=[20])
        bw.append(sync_t() - t0)
    ms_b = float(np.median(bw)) * 1e3
    # batch_test's steps one by one (device synchronised between them): the list cache lookup, the
    # fused score + -inf mask + top-20, the fold-out curves, the users' mean (+ its copy to the host)
    bph = {"lists": [], "score_topk": [], "foldout": [], "mean": []}
    for _ in range(reps):
        t0 = sync_t()
        bl = evaluator._BatchLists.get(users, train_items, test_set, 0, all_users.device)
        t1 = sync_t()
        bidx = bl.route(all_items.shape[0], 20, cfg.d).topk(all_users, all_items, 20, float("-inf"), False)
        t2 = sync_t()
        curves = ops.foldout_metrics(bidx, bl.truth)
        t3 = sync_t()
        ops.column_mean(curves).cpu()
        t4 = sync_t()
        for k_, a_, b_ in (("lists", t0, t1), ("score_topk", t1, t2), ("foldout", t2, t3), ("mean", t3, t4)):
            bph[k_].append((b_ - a_) * 1e3)
    bph = {k_: float(np.median(v)) for k_, v in bph.items()}
    brt = bl.route(all_items.shape[0], 20, cfg.d)
    ms_bk = gpu_ms(lambda: brt.topk(all_users, all_items, 20, float("-inf"), False), reps)
    Eu_h, Ei_h = all_users.float().cpu(), all_items.float().cpu()
    bu = users[:1024]

    def cpu_tf_batch():  # one 1024-user batch: fp32 ratings, -inf train mask, the C++ evaluator restated
        rate = torch.matmul(Eu_h[torch.as_tensor(bu)], Ei_h.t()).numpy()
        for j, x in enumerate(bu):
            rate[j][np.asarray(train_items[x], dtype=np.int64)] = -np.inf
        oracle.eval_score_matrix_foldout(rate, [test_set[x] for x in bu], 20)
    s_b = cpu_s(cpu_tf_batch)
    emit(rows, f"a8 TF batch_test end to end, {cfg.name} shape (evaluator.batch_test)", ms_b, n_test, "test users/s",
         "hbm", 0, len(bu), s_b, f"one 1024-user batch: fp32 torch.matmul ratings + -inf mask + the oracle's C "
                                 f"restatement of the C++ top-K / fold-out evaluator (1 thread), extrapolated",
         CPU_THREADS, f"{n_test} test users on the propagated tables (propagation not included); phases (ms): "
         + ", ".join(f"{k_} {v:.2f}" for k_, v in bph.items()))
    rows[-1]["roofline"] = {"bound": "mfma_f32", "kernel": plan, "launch_ms": ms_bk,
                            "achieved": fl / (ms_bk / 1e3) / 1e12, "peak": F32_PEAK / 1e12, "unit": "TFLOP/s",
                            "frac": fl / (ms_bk / 1e3) / F32_PEAK,
                            "note": "the score + -inf mask + top-20 step of the loop (fused launch + dense route "
                                    "for long masks); the other phases above"}
    rows[-1]["phases_ms"] = bph
    del model, ds, G
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "rows.json"))
    ap.add_argument("--only", default="")
    ap.add_argument("--lib", default=None, help="development: time another liblgx.so build")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    if args.lib:
        _lib.LIB_PATH = os.path.abspath(args.lib)
        _lib._lib = None
        _lib.ALLOW_MISSING = True
    if not torch.cuda.is_available():
        raise SystemExit("bench_rows needs a GPU")
    torch.set_num_threads(CPU_THREADS)
    want = set(x for x in args.only.split(",") if x)
    tmpdir = os.environ.get("TMPDIR", "/tmp")
    steps = [("a2", lambda r: row_a2(r, args.reps)), ("a6", lambda r: row_a6_a9(r, args.reps)),
             ("a10", lambda r: row_a10(r, args.reps)), ("a12", lambda r: row_a12(r, args.reps)),
             ("f1", lambda r: row_f1(r, args.reps)), ("f2", lambda r: row_f2(r, args.reps)),
             ("f2b", lambda r: row_f2b(r, args.reps, tmpdir)),
             ("f3", lambda r: row_f3(r, args.reps, tmpdir)), ("f4", lambda r: row_f4(r, args.reps)),
             ("eval_c1", lambda r: row_eval(r, args.reps, tmpdir, "gowalla")),
             ("eval_c3", lambda r: row_eval(r, args.reps, tmpdir, "amazon"))]
    rows = []
    failed = []
    for name, fn in steps:
        if want and name not in want:
            continue
        try:
            fn(rows)
        except Exception as e:  # report and go on: one row's failure must not hide the others
            print(json.dumps({"row": name, "error": repr(e)}), flush=True)
            failed.append(name)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"device": torch.cuda.get_device_name(0), "rows": rows, "failed": failed}, f, indent=1)
    if failed:
        raise SystemExit(f"rows failed: {failed}")


if __name__ == "__main__":
    main()
