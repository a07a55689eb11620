"""CPU: host-side logic of the package -- launch plans, shard partitioning and column remapping,
ragged-list packing, the synthetic degree law and the Loader's file parsing."""
import numpy as np
import pytest
import torch

from factors_of_serendipity_recommendation_amd.distributed import balanced_bounds, make_shard, pad_table
from factors_of_serendipity_recommendation_amd.graph import CSRGraph, choose_seg_len, make_plan
from factors_of_serendipity_recommendation_amd.ops import lists_to_device_csr
from factors_of_serendipity_recommendation_amd.synth import user_degrees
from oracle import oracle


def _check_plan(indptr, plan):
    lens = np.diff(indptr)
    seen = np.zeros(int(indptr[-1]), dtype=np.int64)
    rows_seen = np.zeros(len(lens), dtype=np.int64)
    for r, part, slot in zip(plan.seg_row, plan.seg_part, plan.seg_slot):
        b = indptr[r] + part * plan.seg_len
        e = indptr[r + 1] if slot < 0 else min(indptr[r + 1], b + plan.seg_len)
        seen[b:e] += 1
        rows_seen[r] += 1
        if slot >= 0:
            assert lens[r] > plan.seg_len
    assert np.all(seen == 1), "every nonzero covered exactly once"
    assert np.all(rows_seen >= 1), "every row (even empty) has a segment"
    # split rows own contiguous slot ranges in part order
    for j, r in enumerate(plan.split_row):
        slots = plan.seg_slot[plan.seg_row == r]
        parts = plan.seg_part[plan.seg_row == r]
        assert np.array_equal(np.sort(slots), np.arange(plan.split_ptr[j], plan.split_ptr[j + 1]))
        assert np.array_equal(slots - plan.split_ptr[j], parts)


@pytest.mark.parametrize("seg_len", [1, 2, 7, 64, 1000])
def test_make_plan_covers_every_nonzero_once(seg_len):
    rng = np.random.default_rng(seg_len)
    lens = rng.zipf(1.5, 400) % 3000
    lens[::17] = 0
    indptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    plan = make_plan(indptr, seg_len)
    _check_plan(indptr, plan)
    # longest-first order
    seg_lens = np.minimum(lens[plan.seg_row] - plan.seg_part * seg_len, seg_len)
    seg_lens = np.where(plan.seg_slot < 0, lens[plan.seg_row], seg_lens)
    assert np.all(np.diff(lens[plan.seg_row]) <= 0)


@pytest.mark.parametrize("seg_len", [1, 7, 64])
def test_make_plan_phases(seg_len):
    """phase-ordered plans (items first, then users): every nonzero once, phases contiguous in
    launch order, longest-first inside each phase; a non-partition is rejected"""
    rng = np.random.default_rng(100 + seg_len)
    lens = rng.zipf(1.5, 300) % 2000
    lens[::13] = 0
    indptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    U = 180
    plan = make_plan(indptr, seg_len, phases=[(U, 300), (0, U)])
    _check_plan(indptr, plan)
    first_user = int(np.argmax(plan.seg_row < U))
    assert np.all(plan.seg_row[:first_user] >= U) and np.all(plan.seg_row[first_user:] < U)
    for sl in (slice(0, first_user), slice(first_user, None)):
        assert np.all(np.diff(lens[plan.seg_row[sl]]) <= 0)
    with pytest.raises(ValueError):
        make_plan(indptr, seg_len, phases=[(0, U), (U + 1, 300)])


def test_choose_seg_len_range():
    assert choose_seg_len(0) == 32
    assert choose_seg_len(1_620_256) == 32    # Gowalla shape
    assert choose_seg_len(5_968_216) == 128   # Amazon-book shape
    assert choose_seg_len(1_000_000_000) == 8192
    assert choose_seg_len(100_000_000) == 4096
    assert choose_seg_len(1 << 24) == 512     # large-graph plans never take the short-segment kernel


def test_balanced_bounds():
    lens = np.array([5, 0, 0, 100, 1, 1, 1, 50, 3, 3])
    indptr = np.concatenate([[0], np.cumsum(lens)])
    for world in (1, 2, 3, 4, 8):
        b = balanced_bounds(indptr, 0, len(lens), world)
        assert b[0] == 0 and b[-1] == len(lens) and np.all(np.diff(b) >= 0) and len(b) == world + 1


def _cpu_graph(U, I, E, seed):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, U, E).astype(np.int32)
    i = rng.integers(0, I, E).astype(np.int32)
    ip, ix, iv = oracle.build_norm_adj(u, i, U, I)
    return CSRGraph(torch.from_numpy(ip), torch.from_numpy(ix), torch.from_numpy(iv), U + I, U + I, U, I), (ip, ix, iv)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_make_shard_pull_and_push_operators(world):
    """Pull rows reproduce the rank's user rows of A X; the push operators' partial sums, added over
    ranks, reproduce every item row; the push operator is the exact transpose (same values)."""
    U, I = 70, 50
    A, (ip, ix, iv) = _cpu_graph(U, I, 900, world)
    X = torch.from_numpy(np.random.default_rng(0).standard_normal((U + I, 4)).astype(np.float32))
    full = oracle.spmm(ip, ix, iv, X.numpy())
    item_sum = None
    for rank in range(world):
        s = make_shard(A, U, I, rank, world, seg_len=8)
        Xi = pad_table(X[U:], s.item_bounds, s.mi)
        yu = oracle.spmm(s.A_pull.indptr.numpy(), s.A_pull.indices.numpy(), s.A_pull.vals.numpy(), Xi.numpy())
        u0, u1 = s.user_bounds[rank], s.user_bounds[rank + 1]
        assert np.allclose(yu, full[u0:u1])
        P = oracle.spmm(s.A_push.indptr.numpy(), s.A_push.indices.numpy(), s.A_push.vals.numpy(),
                        X[u0:u1].numpy())
        assert P.shape == (world * s.mi, 4)
        item_sum = P if item_sum is None else item_sum + P
        dense_pull = np.zeros((s.n_u_local, world * s.mi), np.float32)
        rows = np.repeat(np.arange(s.n_u_local), np.diff(s.A_pull.indptr.numpy()))
        dense_pull[rows, s.A_pull.indices.numpy()] = s.A_pull.vals.numpy()
        dense_push = np.zeros((world * s.mi, s.n_u_local), np.float32)
        rows = np.repeat(np.arange(world * s.mi), np.diff(s.A_push.indptr.numpy()))
        dense_push[rows, s.A_push.indices.numpy()] = s.A_push.vals.numpy()
        assert np.array_equal(dense_push, dense_pull.T)
        assert np.all(np.diff(s.item_bounds) <= s.mi)
    assert np.allclose(item_sum[:I], full[U:], atol=1e-6)
    assert np.all(item_sum[I:] == 0)


def test_lists_to_csr_packing():
    ip, ix = lists_to_device_csr([[5, 1], [], [3]], "cpu")
    assert ip.tolist() == [0, 2, 2, 3] and ix.tolist() == [1, 5, 3]
    ip, ix = lists_to_device_csr([[5, 1]], "cpu", sort=False)
    assert ix.tolist() == [5, 1]


def test_user_degrees_law():
    deg = user_degrees(10000, 500, 200000, 1.0, 0)
    assert deg.min() >= 1 and deg.max() <= 250
    assert abs(int(deg.sum()) - 200000) / 200000 < 0.2


def test_loader_parses_reference_format(tmp_path, mlls):
    from factors_of_serendipity_recommendation_amd.dataloader import Loader
    tp, tx = mlls["train_list_indptr"], mlls["train_list_indices"]
    with open(tmp_path / "train.txt", "w") as f:
        for j, u in enumerate(mlls["train_list_users"]):
            f.write(" ".join(str(x) for x in [u] + list(tx[tp[j]:tp[j + 1]])) + "\n")
    sp_, sx = mlls["test_indptr"], mlls["test_indices"]
    with open(tmp_path / "test.txt", "w") as f:
        for j, u in enumerate(mlls["test_users"]):
            f.write(" ".join(str(x) for x in [u] + list(sx[sp_[j]:sp_[j + 1]])) + "\n")
    ds = Loader(path=str(tmp_path), device="cpu", cache_adj=False)
    assert ds.n_users == int(mlls["n_users"]) and ds.m_items == int(mlls["n_items"])
    assert ds.trainDataSize == len(mlls["train_items"])
    u0 = int(mlls["test_users"][0])
    assert sorted(ds.testDict[u0]) == sorted(sx[sp_[0]:sp_[1]].tolist())
    assert np.array_equal(np.sort(ds.allPos[0]), np.sort(tx[tp[0]:tp[1]]))


def test_bench_measured_traffic_per_call(tmp_path, monkeypatch):
    """bench.measured_traffic: bytes of a committed PMC summary only for the library build that
    made it; with calls_from, every dispatch of the kernels per library call (the seeded scoring
    stages launch the sweep kernel several times per lgx_score_topk call)."""
    import importlib.util
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    (tmp_path / "profiles").mkdir()
    doc = {"lib_sha256_16": "abc", "kernels": {"scoring": {
        "score_topk_bf16_lds": {"hbm_bytes_per_launch": 100e9, "dispatches": 24},
        "score_topk_finalize": {"hbm_bytes_per_launch": 1e9, "dispatches": 6}}}}
    (tmp_path / "profiles" / "r09_cfg_pmc_traffic.json").write_text(json.dumps(doc))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_sha", lambda: "abc")
    ks = ["score_topk_bf16_lds", "score_topk_finalize"]
    gb, src = bench.measured_traffic("cfg", "scoring", 1, ks, calls_from=("score_topk_finalize", 2))
    assert src.endswith("r09_cfg_pmc_traffic.json")
    assert abs(gb - (100 * 24 + 1 * 6) / 3) < 1e-9  # 3 calls: 6 finalize dispatches, 2 per call
    gb1, _ = bench.measured_traffic("cfg", "scoring", 1, ks)
    assert abs(gb1 - 101) < 1e-9                     # per-dispatch means, summed
    monkeypatch.setattr(bench, "lib_sha", lambda: "other")
    assert bench.measured_traffic("cfg", "scoring", 1, ks)[0] is None
    assert bench.measured_traffic("cfg", "scoring", 2, ks)[0] is None


def crafted_extremes(mx: float, mn: float, U: int = 48, I: int = 4000, d: int = 64, seed: int = 0):
    """Embeddings whose f32 scores are exact products u0 * i0: user 0 has u0 = 1 and items 0 / 1
    carry the float16 values of mx / mn, so the score matrix's float16 extremes are exactly them."""
    rng = np.random.default_rng(seed)
    mx16, mn16 = np.float32(np.float16(mx)), np.float32(np.float16(mn))
    eu = np.zeros((U, d), np.float32)
    ei = np.zeros((I, d), np.float32)
    eu[:, 0] = rng.uniform(0.05, 1.0, U).astype(np.float32)
    eu[0, 0] = 1.0
    ei[:, 0] = rng.uniform(mn16, mx16, I).astype(np.float32)
    ei[0, 0], ei[1, 0] = mx16, mn16
    return eu, ei


def test_stratification_bounds_follow_the_pinned_numpy():
    """recommend.py:377-381 under numpy 1.19.5 (environment.yml:253): max_dis and inter are float64
    and inter is rounded to float16 once, at the division.  (9.34, -12.97) is a pair where numpy 2's
    NEP 50 chain of float16 roundings gives another inter (2.24 instead of 2.242) and so other
    labels; the product and the oracle both take the legacy value."""
    from factors_of_serendipity_recommendation_amd import recommend
    mx16, mn16 = np.float16(9.34), np.float16(-12.97)
    legacy = np.float16((float(mx16) + 0.1 - float(mn16)) / 10)        # float64 chain, one rounding
    nep50 = (mx16 + 0.1 - mn16) / 10                                     # float16 chain (numpy >= 2)
    assert legacy == np.float16(2.242) and nep50 == np.float16(2.24) and legacy != nep50
    assert recommend.legacy_float16_bounds(9.34, -12.97, 10, 0.1) == (float(mn16), float(legacy))
    eu, ei = crafted_extremes(9.34, -12.97)
    lab, hist, rmin, rinter = oracle.stratification_labels(eu, ei, [[] for _ in range(len(eu))])
    assert rmin == float(mn16) and rinter == float(legacy)
    s16 = (eu @ ei.T).astype(np.float16)
    assert s16.max() == mx16 and s16.min() == mn16
    assert np.array_equal(lab, np.floor((s16 - mn16) / legacy).astype(np.int8))
    assert (lab != np.floor((s16 - mn16) / nep50).astype(np.int8)).any()  # the pair discriminates


def test_candidate_containers_pickle_as_the_reference_types():
    """CandidateLists pickles as a list of lists (list_res.pickle), CandidateDict as a dict
    (candidate.npy); a CandidateDict row is built once and keeps in-place edits."""
    import pickle
    from factors_of_serendipity_recommendation_amd.recommend import CandidateDict, CandidateLists, _save_object
    picks = np.array([[3, 1, 2], [9, 8, 0]], np.int32)
    lists = CandidateLists(picks, np.array([3, 2], np.int32))
    assert lists == [[3, 1, 2], [9, 8]] and lists[1] == [9, 8] and lists[0:1] == [[3, 1, 2]]
    back = pickle.loads(pickle.dumps(lists))
    assert type(back) is list and back == [[3, 1, 2], [9, 8]]
    d = CandidateDict(lists, [[5], [6, 7]])
    assert dict(d) == {0: [3, 1, 2, 5], 1: [9, 8, 6, 7]} and 2 not in d
    d[0].append(4)
    assert d[0] == [3, 1, 2, 5, 4]
    with pytest.raises(KeyError):
        d[2]
    back = pickle.loads(pickle.dumps(d))
    assert type(back) is dict and back == {0: [3, 1, 2, 5, 4], 1: [9, 8, 6, 7]}


def test_lists_to_csr_sorts_rows_on_the_device_path():
    rng = np.random.default_rng(5)
    lists = [rng.choice(10 ** 6, int(rng.integers(0, 30)), replace=False).tolist() for _ in range(200)]
    ip, ix = lists_to_device_csr(lists, "cpu")
    ip, ix = ip.numpy(), ix.numpy()
    for j, l in enumerate(lists):
        assert ix[ip[j]:ip[j + 1]].tolist() == sorted(l)
    with pytest.raises(ValueError):
        lists_to_device_csr([[1, -2]], "cpu")


@pytest.mark.parametrize("seed", [0, 1])
def test_vectorised_test_one_batch_equals_reference_loops(seed):
    """evaluator.test_one_batch (one membership search for the batch) == the oracle's restatement
    of the reference's per-user loops (Procedure.py:60-72, code/utils.py:218-285), bit for bit:
    ragged truths (1..60 items, duplicates), predictions with hits at any rank, k > |truth|."""
    from factors_of_serendipity_recommendation_amd.evaluator import test_one_batch
    rng = np.random.default_rng(seed)
    n, M = 3000, 5000
    truth = [rng.integers(0, M, int(rng.integers(1, 60))).tolist() for _ in range(n)]
    pred = rng.integers(0, M, (n, 100))
    for i in range(0, n, 3):  # plant hits
        t = truth[i]
        pred[i, rng.integers(0, 100, min(len(t), 5))] = t[:min(len(t), 5)]
    got = test_one_batch(pred, truth, [1, 5, 20, 100])
    ref = oracle.torch_style_metrics(pred, truth, [1, 5, 20, 100])
    for key in ("recall", "precision", "ndcg"):
        assert np.array_equal(got[key], ref[key]), key


@pytest.mark.parametrize("nb", [1, 3, 8])
def test_column_blocks_cover_item_rows_once(nb):
    """CSRGraph.col_blocks: block b of item row r holds exactly the row's nonzeros whose column
    (user id) lies in [b U / nb, (b + 1) U / nb); every block plan covers every item row once
    (global row ids); the user rows' plan is the phased plan's prefix."""
    A, (ip, ix, iv) = _cpu_graph(90, 40, 1500, nb)
    A.plan = None
    A.ensure_plan(8)
    U, I = 90, 40
    blk = A.col_blocks(nb)
    ptr = blk["ptr"].numpy()
    assert ptr.shape == (nb + 1, I)
    cuts = [(b * U) // nb for b in range(nb + 1)]
    for r in range(I):
        row = ip[U + r], ip[U + r + 1]
        for b in range(nb):
            cols = ix[ptr[b, r]:ptr[b + 1, r]]
            assert ((cols >= cuts[b]) & (cols < cuts[b + 1])).all()
        assert ptr[0, r] == row[0] and ptr[nb, r] == row[1]
    for b, pb in enumerate(blk["plans"]):
        lens = np.diff(ptr[b]) if False else ptr[b + 1] - ptr[b]
        ipb = np.concatenate([[0], np.cumsum(lens)])
        pb_local = type(pb)(pb.seg_row - U, pb.seg_part, pb.seg_slot, pb.split_row - U, pb.split_ptr, pb.seg_len)
        _check_plan(ipb, pb_local)
    p = A.plan
    assert (p.seg_row[:blk["n_user_segs"]] < U).all() and (p.seg_row[blk["n_user_segs"]:] >= U).all()
    A.col_block_min, A.col_block_slice = 1, 90 * 4 * 4 // nb + 1
    assert A.col_block_count(4, 4) == nb
    cs = A.c_struct(4, 4)
    assert cs.cb_n == nb and cs.cb_row0 == U and cs.n_segs == blk["n_user_segs"]


def test_test_lists_cache_and_hits_match_get_label():
    """evaluator._TestLists (host-side logic, CPU tensors): reused while the same testDict object
    comes back, rebuilt for a new one; its hit matrix equals utils.getLabel's restatement (_label),
    padding ids (-1) never hit."""
    from factors_of_serendipity_recommendation_amd import evaluator
    rng = np.random.default_rng(4)
    n_items = 300

    class DS:
        def __init__(self):
            self.testDict = {u: sorted(rng.choice(n_items, rng.integers(1, 9), replace=False).tolist())
                             for u in rng.choice(1000, 64, replace=False).tolist()}
            self._pos = {u: sorted(rng.choice(n_items, 5, replace=False).tolist()) for u in self.testDict}

        def getUserPosItems(self, users):
            return [self._pos[u] for u in users]

    ds = DS()
    a = evaluator._TestLists.get(ds, n_items, torch.device("cpu"))
    assert evaluator._TestLists.get(ds, n_items, torch.device("cpu")) is a
    pred = rng.integers(-1, n_items, (len(a.users), 20))
    pred[:, 0] = [ds.testDict[u][0] for u in a.users]  # at least one hit per user
    got = a.hits(torch.from_numpy(pred))
    ref = evaluator._label([ds.testDict[u] for u in a.users], np.maximum(pred, 0)) * (pred >= 0)
    assert np.array_equal(got, ref) and got[:, 0].all()
    ds.testDict = dict(ds.testDict)  # a new object: rebuilt
    assert evaluator._TestLists.get(ds, n_items, torch.device("cpu")) is not a


def test_device_metric_sums_match_host_sums():
    """evaluator._metrics_dev (torch float64, CPU tensors here) equals the host restatement
    _metrics to float64 rounding, users with fewer test items than k included."""
    from factors_of_serendipity_recommendation_amd import evaluator
    rng = np.random.default_rng(9)
    n, K = 3000, 100
    hit = rng.random((n, K)) < 0.05
    recall_n = rng.integers(1, 40, n)
    host = evaluator._metrics(hit.astype(float), recall_n, [1, 5, 20, 100])
    dev = evaluator._metrics_dev(torch.from_numpy(hit), torch.from_numpy(recall_n), [1, 5, 20, 100])
    for key in ("recall", "precision", "ndcg"):
        assert np.allclose(dev[key], host[key], rtol=1e-13, atol=0), key


def test_batch_lists_cache_reuse_and_invalidation():
    """evaluator._BatchLists (CPU tensors): reused for the same dicts and users, rebuilt when the
    users, a dict object or the flag change; flag 1 has no mask and takes the train items as truth."""
    from factors_of_serendipity_recommendation_amd import evaluator
    rng = np.random.default_rng(2)
    train = {u: sorted(rng.choice(500, 6, replace=False).tolist()) for u in range(40)}
    test = {u: sorted(rng.choice(500, 3, replace=False).tolist()) for u in range(40)}
    dev = torch.device("cpu")
    users = list(range(0, 40, 2))
    a = evaluator._BatchLists.get(users, train, test, 0, dev)
    assert evaluator._BatchLists.get(list(users), train, test, 0, dev) is a
    ip, ix = a.mask
    assert ix[ip[1]:ip[2]].tolist() == train[users[1]]
    b = evaluator._BatchLists.get(users[::-1], train, test, 0, dev)
    assert b is not a and b.rows.tolist() == users[::-1]
    c = evaluator._BatchLists.get(users[::-1], dict(train), test, 0, dev)
    assert c is not b
    f1 = evaluator._BatchLists.get(users, train, test, 1, dev)
    tp, tx = f1.truth
    assert f1.mask is None and tx[tp[0]:tp[1]].tolist() == train[users[0]]


def test_eval_caches_see_in_place_edits_and_clear():
    """The evaluator's list caches are rebuilt when a sampled user's list is edited in place (same
    dict object, same length), and clear_caches() drops them."""
    from factors_of_serendipity_recommendation_amd import evaluator
    rng = np.random.default_rng(12)
    n_items = 400

    class DS:
        def __init__(self):
            self.testDict = {u: sorted(rng.choice(n_items, 4, replace=False).tolist()) for u in range(20)}
            self._pos = {u: sorted(rng.choice(n_items, 5, replace=False).tolist()) for u in self.testDict}

        def getUserPosItems(self, users):
            return [self._pos[u] for u in users]

    dev = torch.device("cpu")
    ds = DS()
    a = evaluator._TestLists.get(ds, n_items, dev)
    assert evaluator._TestLists.get(ds, n_items, dev) is a
    ds.testDict[3][-1] = n_items - 1 if ds.testDict[3][-1] != n_items - 1 else 0  # in place, same length
    b = evaluator._TestLists.get(ds, n_items, dev)
    assert b is not a
    ds._pos[5].append(n_items - 2)  # the positives behind the mask change
    c = evaluator._TestLists.get(ds, n_items, dev)
    assert c is not b and evaluator._TestLists.get(ds, n_items, dev) is c
    evaluator.clear_caches()
    assert evaluator._TestLists.get(ds, n_items, dev) is not c

    train = {u: sorted(rng.choice(500, 6, replace=False).tolist()) for u in range(40)}
    test = {u: sorted(rng.choice(500, 3, replace=False).tolist()) for u in range(40)}
    users = list(range(40))
    x = evaluator._BatchLists.get(users, train, test, 0, dev)
    train[0][0] = 499 if train[0][0] != 499 else 498
    y = evaluator._BatchLists.get(users, train, test, 0, dev)
    assert y is not x and evaluator._BatchLists.get(users, train, test, 0, dev) is y
    evaluator.clear_caches()
    assert evaluator._BatchLists.get(users, train, test, 0, dev) is not y


def test_batch_lists_cache_checks_every_user():
    """The batch_test cache compares every user, not a sample: an in-place edit of the caller's user
    list at any position (the same list object), or of an equal numpy array, rebuilds the lists."""
    from factors_of_serendipity_recommendation_amd import evaluator
    rng = np.random.default_rng(21)
    train = {u: sorted(rng.choice(500, 6, replace=False).tolist()) for u in range(300)}
    test = {u: sorted(rng.choice(500, 3, replace=False).tolist()) for u in range(300)}
    dev = torch.device("cpu")
    users = list(range(0, 200))
    a = evaluator._BatchLists.get(users, train, test, 0, dev)
    assert evaluator._BatchLists.get(users, train, test, 0, dev) is a
    for pos in (1, 77, 133, 198):  # positions between the 32 sampled ones included
        users[pos] = 250 + pos % 50
        b = evaluator._BatchLists.get(users, train, test, 0, dev)
        assert b is not a and b.rows.tolist() == users
        a = b
    arr = np.asarray(users, dtype=np.int64)
    c = evaluator._BatchLists.get(arr, train, test, 0, dev)
    assert evaluator._BatchLists.get(arr, train, test, 0, dev) is c
    arr[101] = 299
    assert evaluator._BatchLists.get(arr, train, test, 0, dev).rows.tolist() == arr.tolist()
