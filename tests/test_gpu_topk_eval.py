"""GPU: top-k beyond one wave (k up to 256) and the end-to-end ``Procedure.Test`` against the oracle.

  * lgx_topk_rows / lgx_score_topk for k in (65, 100, 200, 256): the reference's top-k has no
    size limit (tools.h:13-33 partial_sort_copy; torch.topk in Procedure.py:135; TF --Ks up to
    100, LightGCN-tf/utility/parser.py:59).  topk_rows is bit-exact against the oracle (ties ->
    lower index); score_topk gives identical sets modulo ties at 1e-5 of the k-th score.
  * evaluator.Test (Procedure.py:96-174) on mlls, K=3, topks=[20, 100]: the GPU result dict equals
    the oracle restatement = oracle.propagate (f64) -> oracle.score_topk (sigmoid, mask -(1<<10))
    -> oracle.torch_style_metrics (utils.getLabel / RecallPrecision_ATk / NDCGatK_r,
    code/utils.py:218-285) / n_users.  Tolerance: recall / precision equal to 1e-12 (set based);
    NDCG within 1e-6 relative (an exact fp32 tie between two adjacent positions could swap them).
"""
import numpy as np
import pytest
import torch

from oracle import oracle

import factors_of_serendipity_recommendation_amd as lgx
from factors_of_serendipity_recommendation_amd import evaluator, ops

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _bf16_round(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).to(torch.float32).numpy()


def _assert_sets(idx, S, k, rel):
    for r in range(idx.shape[0]):
        g = set(int(x) for x in idx[r] if x >= 0 and np.isfinite(S[r, x]))
        order = np.lexsort((np.arange(S.shape[1]), -S[r]))
        o = [int(x) for x in order[:k] if np.isfinite(S[r, x])]
        if g == set(o):
            continue
        kth = S[r, o[-1]]
        for x in g ^ set(o):
            assert abs(S[r, x] - kth) <= rel * max(1.0, abs(kth)), (r, x, S[r, x], kth)


@pytest.mark.parametrize("k", [65, 100, 128, 200, 256])
@pytest.mark.parametrize("cols", [5000, 40_000])
def test_topk_rows_large_k_bit_exact(k, cols):
    rng = np.random.default_rng(k + cols)
    S = rng.standard_normal((37, cols)).astype(np.float32)
    S[3, :] = 0.5                  # all ties -> lowest indices
    S[4, 100:400] = 9.0            # ties straddling the k-th slot
    idx, val = lgx.topk_rows(torch.from_numpy(S).to(DEV), k)
    oidx, oval = oracle.topk_rows(S, k)
    assert np.array_equal(idx.cpu().numpy(), oidx)
    assert np.array_equal(val.cpu().numpy(), oval)


@pytest.mark.parametrize("k", [1, 20, 64])
@pytest.mark.parametrize("cols", [5000, 100_000, 100_003])
def test_topk_rows_batched_survivors_bit_exact(k, cols):
    """k <= 64: a batch's survivors are packed into one 64-lane merge; a batch with more than 64
    survivors (ascending rows: every value beats the running k-th) merges value by value.  Short
    and long rows, float4 and scalar loads, ties and infinities, bit-exact against the oracle."""
    rng = np.random.default_rng(3 * k + cols)
    S = rng.standard_normal((24, cols)).astype(np.float32)
    S[1] = np.arange(cols, dtype=np.float32)            # ascending: every batch overflows 64
    S[2] = -np.arange(cols, dtype=np.float32)           # descending: no event after the first batch
    S[3] = 0.25                                         # all ties -> lowest indices
    S[4, ::97] = 7.0                                    # spread ties above everything else
    S[5, cols // 2:] = np.inf                           # infinities
    S[6] = -np.inf
    S[7, -70:] = 50.0                                   # the best values in the last batch
    idx, val = lgx.topk_rows(torch.from_numpy(S).to(DEV), k)
    oidx, oval = oracle.topk_rows(S, k)
    assert np.array_equal(idx.cpu().numpy(), oidx)
    assert np.array_equal(val.cpu().numpy(), oval)


@pytest.mark.parametrize("dtype,d", [(torch.float32, 64), (torch.bfloat16, 128), (torch.bfloat16, 256)])
@pytest.mark.parametrize("k", [65, 100, 200])
def test_score_topk_large_k_masked(dtype, d, k):
    """k > 64: the register-fragment kernel (4 waves per workgroup up to k = 128, 1 above) and the
    two- / four-register finalize merge; small batches split the catalog so several partial lists
    per user are merged."""
    rng = np.random.default_rng(7 * k + d)
    B, I = 150, 6000
    Q = rng.standard_normal((B, d)).astype(np.float32)
    items = rng.standard_normal((I, d)).astype(np.float32)
    if dtype == torch.bfloat16:
        Q, items = _bf16_round(Q), _bf16_round(items)
    masks = [np.unique(rng.integers(0, I, rng.integers(0, 80))) for _ in range(B)]
    mask = ops.lists_to_device_csr(masks, DEV)
    idx, val = lgx.score_topk(torch.from_numpy(Q).to(DEV).to(dtype), torch.from_numpy(items).to(DEV).to(dtype), k,
                              mask=mask)
    S = Q.astype(np.float64) @ items.astype(np.float64).T
    for u, m in enumerate(masks):
        S[u, m] = -np.inf
    idx = idx.cpu().numpy()
    _assert_sets(idx, S, k, 1e-5)
    assert all(len(set(r)) == k for r in idx.tolist())
    got = np.take_along_axis(S, idx.astype(np.int64), 1)
    assert np.allclose(val.cpu().numpy(), got, rtol=1e-5, atol=1e-5)
    assert (np.diff(val.cpu().numpy(), axis=1) <= 0).all()  # descending


def test_score_topk_large_k_masked_tail():
    """k = 100 over a 90-item catalog with masks: the masked tail fills slots in index order and slots
    past the catalog are -1, as for k <= 64."""
    rng = np.random.default_rng(5)
    Q = torch.from_numpy(rng.standard_normal((4, 32)).astype(np.float32)).to(DEV)
    items = torch.from_numpy(rng.standard_normal((90, 32)).astype(np.float32)).to(DEV)
    masks = [list(range(0, 90, 3)), [], list(range(90)), [5, 6]]
    mask = ops.lists_to_device_csr(masks, DEV)
    idx, val = lgx.score_topk(Q, items, 100, mask=mask, mask_value=-1024.0, apply_sigmoid=True)
    oidx, oval = oracle.score_topk(Q.cpu().numpy(), items.cpu().numpy(), 100, masks, mask_value=-1024.0,
                                   apply_sigmoid=True)
    assert np.array_equal(idx.cpu().numpy(), oidx)
    assert np.allclose(val.cpu().numpy(), oval, rtol=1e-6, atol=1e-7)


def _mlls_loader(mlls, tmp_path):
    from factors_of_serendipity_recommendation_amd.dataloader import Loader
    tp, tx = mlls["train_list_indptr"], mlls["train_list_indices"]
    with open(tmp_path / "train.txt", "w") as f:
        for j, u in enumerate(mlls["train_list_users"]):
            f.write(" ".join(str(x) for x in [u] + list(tx[tp[j]:tp[j + 1]])) + "\n")
    sp_, sx = mlls["test_indptr"], mlls["test_indices"]
    with open(tmp_path / "test.txt", "w") as f:
        for j, u in enumerate(mlls["test_users"]):
            f.write(" ".join(str(x) for x in [u] + list(sx[sp_[j]:sp_[j + 1]])) + "\n")
    return Loader(path=str(tmp_path), device=DEV)


@pytest.mark.parametrize("topks,d", [([20, 100], 64), ([20], 64), ([5, 20], 128)])
def test_procedure_test_matches_oracle_restatement(mlls, tmp_path, topks, d):
    """evaluator.Test == Procedure.Test restated by the oracle on the mlls graph: the shipped d = 64
    embeddings at k = 100 (the register-fragment kernel) and k = 20 (the fp32 LDS walk, 8 staggered
    waves, catalog split), and random d = 128 embeddings at k = 20 (the same walk at d = 128)."""
    from factors_of_serendipity_recommendation_amd.model import LightGCN
    ds = _mlls_loader(mlls, tmp_path)
    eu, ei = mlls["emb_user"].astype(np.float32), mlls["emb_item"].astype(np.float32)
    if d != eu.shape[1]:
        rng = np.random.default_rng(d)
        eu = (rng.standard_normal((eu.shape[0], d)) * 0.1).astype(np.float32)
        ei = (rng.standard_normal((ei.shape[0], d)) * 0.1).astype(np.float32)
    plan = ops.score_topk_plan(len(ds.testDict), ei.shape[0], d, torch.float32, max(topks))
    assert plan.startswith("score_topk_f32_lds<8 waves") == (max(topks) <= 32), plan
    cfg = {"latent_dim_rec": eu.shape[1], "lightGCN_n_layers": 3, "keep_prob": 0.6, "A_split": False,
           "pretrain": 1, "user_emb": eu, "item_emb": ei, "dropout": 0}
    model = LightGCN(cfg, ds).to(DEV)
    got = evaluator.Test(ds, model, topks=topks)

    # oracle: Procedure.Test restated on the CPU (f64 propagation of the same adjacency)
    A = ds.getSparseGraph().coalesce().cpu()
    idx = A.indices().numpy()
    U, I = ds.n_users, ds.m_items
    ip = np.zeros(U + I + 1, dtype=np.int64)
    np.add.at(ip, idx[0] + 1, 1)
    ip = np.cumsum(ip)
    prop = oracle.propagate(ip, idx[1].astype(np.int32), A.values().numpy().astype(np.float32),
                            np.concatenate([eu, ei]), 3)
    users = list(ds.testDict.keys())
    allPos = ds.getUserPosItems(users)
    oidx, _ = oracle.score_topk(prop[:U][users].astype(np.float32), prop[U:].astype(np.float32), max(topks),
                                [list(p) for p in allPos], mask_value=-float(1 << 10), apply_sigmoid=True)
    truth = [ds.testDict[u] for u in users]
    ref = oracle.torch_style_metrics(oidx, truth, topks)
    for key in ("recall", "precision"):
        assert np.allclose(got[key], ref[key] / len(users), rtol=0, atol=1e-12), (key, got[key], ref[key])
    assert np.allclose(got["ndcg"], ref["ndcg"] / len(users), rtol=1e-6, atol=0), (got["ndcg"], ref["ndcg"])
    assert got["recall"][-1] >= got["recall"][0] > 0


@pytest.mark.parametrize("d", [64, 128])
def test_dense_masked_route_matches_float64(d):
    """ops.score_topk_dense_masked (the evaluator's route for users with long masks: dense raw scores,
    masked entries -inf, row top-k) returns k distinct unmasked items, each within 1e-5 of the exact
    k-th best unmasked score, for masks of 65..3000 items; chunked over users."""
    g = torch.Generator(device=DEV).manual_seed(d)
    B, I, k = 300, 20_000, 20
    Q = torch.randn(B + 50, d, device=DEV, generator=g) / 8
    items = torch.randn(I, d, device=DEV, generator=g) / 8
    rows = torch.randperm(B + 50, device=DEV, generator=g)[:B]
    lens = torch.randint(65, 3000, (B,), generator=torch.Generator().manual_seed(d)).tolist()
    # each user's best items masked first, so the mask hits the scores that matter
    S = Q[rows].double() @ items.double().T
    order = torch.argsort(S, dim=1, descending=True)
    lists = [sorted(order[u, :lens[u]].tolist()) for u in range(B)]
    mask = ops.lists_to_device_csr(lists, DEV)
    idx = ops.score_topk_dense_masked(Q, items, k, rows, mask, chunk_bytes=64 * I * 4)
    for u in range(B):
        S[u, torch.tensor(lists[u], device=DEV)] = float("-inf")
    kth = torch.topk(S, k, dim=1).values[:, -1:]
    got = S.gather(1, idx.long())
    assert torch.isfinite(got).all(), "a masked item was returned"
    assert (got >= kth - 1e-5 * kth.abs().clamp(min=1.0)).all()
    srt = idx.long().sort(1).values
    assert (srt[:, 1:] != srt[:, :-1]).all()


def test_evaluator_route_splits_long_masks():
    """evaluator._Route: users with more than dense_mask_min(I, d) masked items (and at least k unmasked)
    go to the dense route, the rest to the fused launch; both results land in set order and agree
    with the fused launch over everyone as top-k sets."""
    from factors_of_serendipity_recommendation_amd.evaluator import _Route, dense_mask_min
    g = torch.Generator(device=DEV).manual_seed(3)
    B, I, d, k = 2000, 30_000, 64, 20
    Q = torch.randn(B, d, device=DEV, generator=g) / 8
    items = torch.randn(I, d, device=DEV, generator=g) / 8
    rng = np.random.default_rng(3)
    thr = dense_mask_min(I, d)
    lens = np.where(rng.random(B) < 0.1, rng.integers(thr + 1, 5000, B), rng.integers(0, 40, B))
    lens[7] = I - k + 1  # fewer than k unmasked items: stays on the fused path (its masked tail)
    lists = [sorted(rng.choice(I, int(n), replace=False).tolist()) for n in lens]
    mask = ops.lists_to_device_csr(lists, DEV)
    rows = torch.arange(B, device=DEV)
    r = _Route(rows, mask, I, k, d)
    assert r.thr == thr and r.n_heavy == int(((lens > thr) & (lens <= I - k)).sum()) > 0
    idx = r.topk(Q, items, k, float("-inf"), False)
    ref, _ = ops.score_topk(Q, items, k, mask=mask)
    S = Q.double() @ items.double().T
    for u in range(B):
        if lists[u]:
            S[u, torch.tensor(lists[u], device=DEV)] = float("-inf")
    kth = torch.topk(S, k, dim=1).values[:, -1:]
    got = S.gather(1, idx.long())
    heavy = torch.from_numpy((lens > thr) & (lens <= I - k)).to(DEV)
    assert torch.isfinite(got[heavy]).all()
    assert (got[heavy] >= (kth - 1e-5 * kth.abs().clamp(min=1.0))[heavy]).all()
    assert torch.equal(idx[~heavy], ref[~heavy])  # the light users are the fused launch's own result


@pytest.mark.parametrize("topks", [[20], [1, 5, 20], [20, 5], [100, 10, 50],
                                   [1, 2, 3, 5, 8, 10, 15, 20, 30, 40, 50]])
def test_test_metrics_kernel_matches_host_restatement(topks):
    """lgx_test_metrics (Procedure.Test's getLabel + RecallPrecision_ATk + NDCGatK_r sums in one launch)
    against the host restatement of utils.py:218-285 on the same rankings: short and power-law test
    lists (binary search over thousands of items), duplicated test items (len() counts them, a hit
    does not), rankings padded with -1, several topks in any order.  float64 sums in another order:
    1e-12 relative."""
    rng = np.random.default_rng(len(topks) * 7 + max(topks))
    n_users, n_items, K = 3000, 20000, max(topks)
    lens = np.minimum(rng.zipf(1.6, n_users), 5000)
    truths = [list(rng.choice(n_items, size=int(L), replace=False)) for L in lens]
    for u in range(0, n_users, 37):  # duplicates
        if truths[u]:
            truths[u] = truths[u] + truths[u][:2]
    rank = np.stack([rng.choice(n_items, size=K, replace=False) for _ in range(n_users)]).astype(np.int32)
    for u in range(n_users):  # plant hits at random ranks
        t = truths[u]
        for j in rng.choice(K, size=min(len(t), int(rng.integers(0, 6))), replace=False):
            rank[u, j] = t[int(rng.integers(0, len(t)))]
    rank[::53, -3:] = -1
    # a ranking must not repeat an item (getLabel counts each position): drop planted repeats
    for u in range(n_users):
        _, first = np.unique(rank[u], return_index=True)
        dup = np.setdiff1d(np.arange(K), first)
        rank[u, dup] = -1
    recall_n = np.array([len(t) for t in truths], dtype=np.int64)
    hit = np.array([[x in set(t) for x in rank[u]] for u, t in enumerate(truths)], dtype=float)
    want = evaluator._metrics(hit, recall_n, topks)
    truth = ops.lists_to_device_csr([sorted(set(t)) for t in truths], DEV, sort=True)
    got = ops.test_metrics(torch.from_numpy(rank).to(DEV), truth, topks,
                           torch.from_numpy(recall_n).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(got[0], want["recall"], rtol=1e-12)
    np.testing.assert_allclose(got[1] / np.asarray(topks, dtype=float), want["precision"], rtol=1e-12)
    np.testing.assert_allclose(got[2], want["ndcg"], rtol=1e-12)


def test_test_metrics_c_abi_layout_is_topk_major():
    """lgx_test_metrics through the C ABI (as a C caller following include/lgx.h binds it), 2 topks:
    sums[3*t + m] = metric m (recall, right, ndcg) of topks[t], i.e. [n_topks, 3]."""
    import ctypes
    from factors_of_serendipity_recommendation_amd import _lib
    rng = np.random.default_rng(11)
    n_users, n_items, topks = 500, 2000, [5, 20]
    K = max(topks)
    truths = [sorted(set(rng.choice(n_items, size=int(rng.integers(1, 40)), replace=False).tolist()))
              for _ in range(n_users)]
    rank = np.stack([rng.choice(n_items, size=K, replace=False) for _ in range(n_users)]).astype(np.int32)
    for u in range(n_users):
        rank[u, int(rng.integers(0, K))] = truths[u][0] if truths[u][0] not in rank[u] else rank[u, 0]
    ip, ix = ops.lists_to_device_csr(truths, DEV, sort=True)
    r = torch.from_numpy(rank).to(DEV)
    tk = torch.tensor(topks, dtype=torch.int32, device=DEV)
    tl = ops.inv_log2_table(K, DEV)
    L = _lib.lib()
    ws = ctypes.c_size_t(0)
    _lib.check(L.lgx_test_metrics_workspace(n_users, len(topks), ctypes.byref(ws)), "ws")
    work = torch.empty(max(ws.value, 8), dtype=torch.uint8, device=DEV)
    sums = torch.full((len(topks) * 3,), float("nan"), dtype=torch.float64, device=DEV)
    _lib.check(L.lgx_test_metrics(r.data_ptr(), n_users, K, ip.data_ptr(), ix.data_ptr(), None, tk.data_ptr(),
                                  len(topks), tl.data_ptr(), sums.data_ptr(), work.data_ptr(), ws.value, None),
               "lgx_test_metrics")
    torch.cuda.synchronize()
    got = sums.cpu().numpy().reshape(len(topks), 3)
    hit = np.array([[x in set(t) for x in rank[u]] for u, t in enumerate(truths)], dtype=float)
    want = evaluator._metrics(hit, np.array([len(t) for t in truths]), topks)
    for t, k in enumerate(topks):
        np.testing.assert_allclose(got[t], [want["recall"][t], want["precision"][t] * k, want["ndcg"][t]],
                                   rtol=1e-12)
