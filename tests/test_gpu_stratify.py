"""GPU: stratified candidate sets (recommend.py:314-452).  Labels and histograms against the numpy
restatement (float16 arithmetic); the random picks by their exact per-label quotas, membership and
seed determinism -- the reference draws with pandas' global numpy generator, so the picks match in
distribution, not in bits (parity unpinned beyond these properties)."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle
from factors_of_serendipity_recommendation_amd import _lib, ops, recommend

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _setup(seed=0, U=40, I=3000, d=32):
    rng = np.random.default_rng(seed)
    eu = (rng.standard_normal((U, d)) * 0.4).astype(np.float32)
    ei = (rng.standard_normal((I, d)) * 0.4).astype(np.float32)
    train = [np.sort(rng.choice(I, int(rng.integers(5, 80)), replace=False)).tolist() for _ in range(U)]
    return eu, ei, train


def _labels(eu, ei, train, num_fold=10):
    Eu, Ei = torch.from_numpy(eu).to(DEV), torch.from_numpy(ei).to(DEV)
    min16, inter16 = recommend.stratification_bounds(Eu, Ei, num_fold, 0.1)
    mp, mi = ops.lists_to_device_csr(train, DEV)
    S = ops.score_dense(Eu, Ei)
    U, I = S.shape
    lab = torch.empty((U, I), dtype=torch.int8, device=DEV)
    hist = torch.empty((U, num_fold + 1), dtype=torch.int32, device=DEV)
    _lib.check(_lib.lib().lgx_strat_labels(S.data_ptr(), U, I, min16, inter16, num_fold, mp.data_ptr(), mi.data_ptr(),
                                           lab.data_ptr(), hist.data_ptr(), None), "lgx_strat_labels")
    torch.cuda.synchronize()
    return lab, hist, min16, inter16


def _select(lab, hist, targets, seed, n_bins=11, stride=None, flags=0):
    U, I = lab.shape
    stride = stride or int(max(targets))
    out = torch.empty((U, stride), dtype=torch.int32, device=DEV)
    cnt = torch.empty(U, dtype=torch.int32, device=DEV)
    tgt = torch.as_tensor(np.asarray(targets, dtype=np.int32), device=DEV)
    _lib.check(_lib.lib().lgx_strat_select_ex(lab.data_ptr(), U, I, hist.data_ptr(), n_bins, tgt.data_ptr(), seed,
                                              out.data_ptr(), stride, cnt.data_ptr(), flags, None),
               "lgx_strat_select_ex")
    return out.cpu().numpy(), cnt.cpu().numpy()


def test_labels_and_histograms_match_restatement():
    eu, ei, train = _setup()
    lab, hist, min16, inter16 = _labels(eu, ei, train)
    rlab, rhist, rmin, rinter = oracle.stratification_labels(eu, ei, train)
    assert min16 == rmin and inter16 == rinter
    lab = lab.cpu().numpy()
    diff = lab != rlab
    # only fp32 dot-order differences right at a float16 boundary may flip a label, by one
    assert diff.mean() < 1e-3 and (np.abs(lab.astype(int) - rlab.astype(int))[diff] <= 1).all()
    assert (lab[rlab == -1] == -1).all()
    assert np.abs(hist.cpu().numpy() - rhist).sum() <= 2 * diff.sum()


@pytest.mark.parametrize("K", [1, 37, 200, 1000])
def test_selection_quotas_membership_and_determinism(K):
    eu, ei, train = _setup(1)
    lab, hist, _, _ = _labels(eu, ei, train)
    L, H = lab.cpu().numpy(), hist.cpu().numpy()
    out, cnt = _select(lab, hist, [K] * len(train), seed=5)
    out2, cnt2 = _select(lab, hist, [K] * len(train), seed=5)
    out3, _ = _select(lab, hist, [K] * len(train), seed=6)
    assert np.array_equal(out, out2) and np.array_equal(cnt, cnt2)
    assert not np.array_equal(out, out3)
    for u in range(len(train)):
        q = oracle.stratification_quotas(H[u], K)
        n = int(q.sum())
        picks = out[u, :cnt[u]]
        expect = K if n >= K else min(K, 2 * n)
        assert cnt[u] == expect
        first = picks[:min(n, K)]
        assert len(set(first.tolist())) == len(first)  # distinct
        assert not np.isin(first, train[u]).any()
        if n <= K:  # nothing trimmed: every quota met exactly
            assert np.array_equal(np.bincount(L[u, first], minlength=len(q)), q)
        if cnt[u] > n:  # sample_list padding re-draws from the list itself
            assert np.isin(picks[n:], first).all()


def test_selection_is_uniform_within_a_label():
    rng = np.random.default_rng(3)
    U, I = 1, 400
    lab = torch.zeros((U, I), dtype=torch.int8, device=DEV)  # one label, every item eligible
    hist = torch.tensor([[I] + [0] * 10], dtype=torch.int32, device=DEV)
    counts = np.zeros(I)
    for s in range(300):
        out, cnt = _select(lab, hist, [40], seed=int(rng.integers(1, 2 ** 62)))
        counts[out[0, :cnt[0]]] += 1
    expected = 300 * 40 / I
    chi2 = ((counts - expected) ** 2 / expected).sum()
    assert chi2 < (I - 1) + 6 * np.sqrt(2 * (I - 1)), chi2


def test_create_candidates_stratification_dropin(tmp_path):
    import pandas as pd
    eu, ei, train = _setup(2, U=30, I=2000)
    rng = np.random.default_rng(9)
    test = [rng.choice(2000, 3, replace=False).tolist() for _ in range(30)]
    root = tmp_path / "data"
    (root / "s").mkdir(parents=True)
    np.save(root / "s" / "emb_user.npy", eu)
    np.save(root / "s" / "emb_item.npy", ei)
    for name, lists in (("rating_train.csv", train), ("rating_test.csv", test)):
        pd.DataFrame([(u, i) for u, l in enumerate(lists) for i in l], columns=["userInd", "itemInd"]) \
            .to_csv(root / "s" / name, index=False)
    cand = recommend.create_candidates_stratification("s", 3, K_c=300, data_root=str(root), device=DEV)
    assert sorted(cand) == list(range(30))
    for u in range(30):
        assert len(cand[u]) == 300 and cand[u][-3:] == test[u]
        assert not np.isin(cand[u][:-3], train[u]).any()
    assert os.path.exists(root / "s" / "rec" / "3" / "candidate.npy")


def test_create_candidates_groups_targets_and_bounds(tmp_path, monkeypatch):
    """Train user ids that are not dense 0..n-1 and more emb_user rows than train groups: the
    reference zips mat_label row j (user j) with the j-th train group, takes the target from the
    group key's test list (recommend.py:421,426), appends the test list of position j (:450), and
    its label grid spans every emb_user row (np.max / np.min of the full product, :375-377)."""
    import pandas as pd
    U, I, K_c = 30, 2000, 300
    eu, ei, train = _setup(4, U=U, I=I)
    eu[U - 1] *= 6.0  # the last user (no train group) holds the extreme scores
    rng = np.random.default_rng(10)
    test = [rng.choice(I, int(rng.integers(1, 6)), replace=False).tolist() for _ in range(U)]
    groups = [u for u in range(U - 1) if u != 4]  # user 4 and the last user have no train rows
    root = tmp_path / "data"
    (root / "s").mkdir(parents=True)
    np.save(root / "s" / "emb_user.npy", eu)
    np.save(root / "s" / "emb_item.npy", ei)
    pd.DataFrame([(u, i) for u in groups for i in train[u]], columns=["userInd", "itemInd"]) \
        .to_csv(root / "s" / "rating_train.csv", index=False)
    pd.DataFrame([(u, i) for u, l in enumerate(test) for i in l], columns=["userInd", "itemInd"]) \
        .to_csv(root / "s" / "rating_test.csv", index=False)
    seen = {}
    real = recommend.stratified_candidates

    def spy(*args, **kw):
        seen["bounds"] = kw.get("bounds")
        seen["n"] = args[0].shape[0]
        return real(*args, **kw)

    monkeypatch.setattr(recommend, "stratified_candidates", spy)
    cand = recommend.create_candidates_stratification("s", 3, K_c=K_c, data_root=str(root), device=DEV)
    full = recommend.stratification_bounds(torch.from_numpy(eu).to(DEV), torch.from_numpy(ei).to(DEV), 10, 0.1)
    sub = recommend.stratification_bounds(torch.from_numpy(eu[:len(groups)]).to(DEV), torch.from_numpy(ei).to(DEV),
                                          10, 0.1)
    assert seen["n"] == len(groups) and seen["bounds"] == full and full != sub
    assert sorted(cand) == list(range(len(groups)))
    for j, g in enumerate(groups):
        assert len(cand[j]) == K_c - len(test[g]) + len(test[j]), j
        assert cand[j][len(cand[j]) - len(test[j]):] == test[j]
        assert not np.isin(cand[j][:K_c - len(test[g])], train[g]).any()


def test_fast_select_equals_radix_select():
    """the cut-and-rank fast path picks exactly the sets (and order) of the exact radix select:
    long rows (fast path taken), a tiny label (cut = everything), and a row whose candidates
    overflow the fast path's buffer (falls back inside the same launch)"""
    rng = np.random.default_rng(21)
    U, I = 6, 48_000
    lab_h = rng.integers(0, 11, (U, I)).astype(np.int8)
    lab_h[:, rng.choice(I, 500, replace=False)] = -1          # train items
    lab_h[1, :] = np.where(lab_h[1] >= 0, 3, -1)              # one label only
    lab_h[2, rng.choice(I, 7, replace=False)] = 10            # label 10 nearly empty in row 2
    lab_h[2, lab_h[2] == 10] = 9
    lab_h[2, :7] = 10
    hist_h = np.stack([np.bincount(r[r >= 0], minlength=11) for r in lab_h]).astype(np.int32)
    lab = torch.from_numpy(lab_h).to(DEV)
    hist = torch.from_numpy(hist_h).to(DEV)
    targets = [1000, 1000, 900, 37, 1024, 1]
    fast = _select(lab, hist, targets, seed=12345, stride=1024)
    exact = _select(lab, hist, targets, seed=12345, stride=1024, flags=_lib.LGX_STRAT_EXACT)
    assert np.array_equal(fast[1], exact[1])
    for u in range(U):
        assert np.array_equal(fast[0][u, :fast[1][u]], exact[0][u, :exact[1][u]])


@pytest.mark.parametrize("dtype,d,I,F", [(torch.float32, 64, 4096, 10), (torch.float32, 40, 3001, 10),
                                         (torch.float32, 128, 3001, 16), (torch.float32, 256, 1030, 10),
                                         (torch.bfloat16, 128, 4096, 10), (torch.bfloat16, 256, 2999, 10),
                                         (torch.float32, 64, 3001, 24)])
def test_fused_labels_equal_two_step_labels(dtype, d, I, F):
    """lgx_strat_labels_fused (scores labelled and counted in the MFMA epilogue; > 16 folds count
    in a separate pass) == lgx_score_dense + lgx_strat_labels, label for label and count for count,
    masked items included; tails where the catalog is not a multiple of 4 / 16; 300 users = one
    full and one partial 256-user group."""
    eu, ei, train = _setup(seed=d + I, U=300, I=I, d=d)
    Eu, Ei = torch.from_numpy(eu).to(DEV).to(dtype), torch.from_numpy(ei).to(DEV).to(dtype)
    min16, inter16 = recommend.stratification_bounds(Eu.float(), Ei.float(), F, 0.1)
    mp, mi = ops.lists_to_device_csr(train, DEV)
    assert recommend.fused_labels_eligible(Eu, d)
    lab_f, hist_f = recommend.strat_labels(Eu, Ei, mp, mi, min16, inter16, F, fused=True)
    lab_2, hist_2 = recommend.strat_labels(Eu, Ei, mp, mi, min16, inter16, F, fused=False)
    assert torch.equal(lab_f, lab_2)
    assert torch.equal(hist_f, hist_2)
    assert (lab_f >= -1).all() and (lab_f <= F).all()


def test_fused_stratified_candidates_equal_two_step():
    eu, ei, train = _setup(seed=5, U=700, I=5000, d=64)
    Eu, Ei = torch.from_numpy(eu).to(DEV), torch.from_numpy(ei).to(DEV)
    targets = [300] * len(train)
    a = recommend.stratified_candidates(Eu, Ei, train, targets, seed=3, batch=256, fused=True)
    b = recommend.stratified_candidates(Eu, Ei, train, targets, seed=3, batch=256, fused=False)
    assert a == b


def test_stratified_candidates_pipelined_batches_equal_per_batch_select():
    """stratified_candidates overlaps the host unpacking of batch b with batch b+1 on the GPU: the
    lists equal a synchronous per-batch labels + select with the same per-batch seeds, in order,
    over 3 batches (the last partial) and varied per-user targets."""
    eu, ei, train = _setup(seed=9, U=600, I=4000, d=64)
    Eu, Ei = torch.from_numpy(eu).to(DEV), torch.from_numpy(ei).to(DEV)
    rng = np.random.default_rng(2)
    targets = rng.integers(50, 400, len(train)).tolist()
    got = recommend.stratified_candidates(Eu, Ei, train, targets, seed=7, batch=256)
    min16, inter16 = recommend.stratification_bounds(Eu, Ei, 10, 0.1)
    mp, mi = ops.lists_to_device_csr(train, DEV, sort=True)
    K = max(targets)
    want = []
    for b0 in range(0, len(train), 256):
        b1 = min(len(train), b0 + 256)
        lab, hist = recommend.strat_labels(Eu[b0:b1], Ei, mp[b0:], mi, min16, inter16, 10, None)
        o, c = _select(lab, hist, targets[b0:b1], seed=(7 * 0x9E3779B97F4A7C15 + b0) % 2 ** 64, stride=K)
        want.extend(o[j, :c[j]].tolist() for j in range(b1 - b0))
    assert len(got) == len(train)
    assert got == want


@pytest.mark.parametrize("fused", [True, False])
def test_labels_on_a_pair_where_numpy_versions_disagree(fused):
    """(max, min) = (9.34, -12.97) in float16: the reference's numpy 1.19 forms inter = 2.242
    (float64 chain rounded once), numpy 2's NEP 50 chain 2.24.  Scores are exact products, so the
    GPU labels (fused epilogue and two-step) must equal the legacy-numpy oracle label for label."""
    from test_host_logic import crafted_extremes
    eu, ei = crafted_extremes(9.34, -12.97, U=300, I=5000)
    rng = np.random.default_rng(4)
    train = [np.sort(rng.choice(5000, 20, replace=False)).tolist() for _ in range(300)]
    Eu, Ei = torch.from_numpy(eu).to(DEV), torch.from_numpy(ei).to(DEV)
    min16, inter16 = recommend.stratification_bounds(Eu, Ei, 10, 0.1)
    assert np.float16(inter16) == np.float16(2.242)
    rlab, rhist, rmin, rinter = oracle.stratification_labels(eu, ei, train)
    assert (min16, inter16) == (rmin, rinter)
    mp, mi = ops.lists_to_device_csr(train, DEV)
    lab, hist = recommend.strat_labels(Eu, Ei, mp, mi, min16, inter16, 10, fused=fused)
    assert np.array_equal(lab.cpu().numpy(), rlab)
    assert np.array_equal(hist.cpu().numpy(), rhist)


def _write_dataset(root, eu, ei, train, test):
    import pandas as pd
    (root / "s").mkdir(parents=True, exist_ok=True)
    np.save(root / "s" / "emb_user.npy", eu)
    np.save(root / "s" / "emb_item.npy", ei)
    for name, lists in (("rating_train.csv", train), ("rating_test.csv", test)):
        pd.DataFrame([(u, i) for u, l in enumerate(lists) for i in l], columns=["userInd", "itemInd"]) \
            .to_csv(root / "s" / name, index=False)


def test_create_candidates_honours_the_reference_caches(tmp_path):
    """recommend.py:365-368: candidate.npy with one entry per user is returned as is; :416-440:
    list_res.pickle is written by the first call and, when present, replaces the sampling."""
    import pickle
    eu, ei, train = _setup(2, U=30, I=2000)
    rng = np.random.default_rng(9)
    test = [rng.choice(2000, 3, replace=False).tolist() for _ in range(30)]
    root = tmp_path / "data"
    _write_dataset(root, eu, ei, train, test)
    rec = root / "s" / "rec" / "3"
    first = recommend.create_candidates_stratification("s", 3, K_c=300, data_root=str(root), device=DEV)
    assert isinstance(first, recommend.CandidateDict)
    with open(rec / "list_res.pickle", "rb") as f:
        list_res = pickle.load(f)
    assert type(list_res) is list and all(type(r) is list for r in list_res)
    assert [r + test[u] for u, r in enumerate(list_res)] == [first[u] for u in range(30)]
    saved = np.load(rec / "candidate.npy", allow_pickle=True).item()
    assert type(saved) is dict and saved == dict(first)
    # candidate.npy present with one entry per user -> returned without recomputing
    np.save(rec / "candidate.npy", {u: [u] for u in range(30)})
    assert recommend.create_candidates_stratification("s", 3, K_c=300, data_root=str(root), device=DEV) == \
        {u: [u] for u in range(30)}
    # wrong length -> ignored; list_res.pickle present -> its lists + the test items
    np.save(rec / "candidate.npy", {0: [1]})
    with open(rec / "list_res.pickle", "wb") as f:
        pickle.dump([[7, 8]] * 30, f)
    again = recommend.create_candidates_stratification("s", 3, K_c=300, data_root=str(root), device=DEV)
    assert all(again[u] == [7, 8] + test[u] for u in range(30))
    assert np.load(rec / "candidate.npy", allow_pickle=True).item() == dict(again)


def test_create_candidates_raises_where_the_reference_raises(tmp_path):
    """KeyError for a user without test items (recommend.py:426); ValueError when K_c - |test| is
    negative (DataFrame.sample(n < 0)) or more than sample_list can pad (random.sample, :317)."""
    eu, ei, train = _setup(2, U=10, I=500)
    rng = np.random.default_rng(1)
    test = [rng.choice(500, 3, replace=False).tolist() for _ in range(10)]
    root = tmp_path / "a"
    _write_dataset(root, eu, ei, train, test[:9] + [[]])
    with pytest.raises(KeyError):
        recommend.create_candidates_stratification("s", 1, K_c=50, data_root=str(root), device=DEV)
    root = tmp_path / "b"
    _write_dataset(root, eu, ei, train, test)
    with pytest.raises(ValueError):
        recommend.create_candidates_stratification("s", 1, K_c=2, data_root=str(root), device=DEV)
    Eu, Ei = torch.from_numpy(eu).to(DEV), torch.from_numpy(ei).to(DEV)
    n_free = [500 - len(t) for t in train]
    with pytest.raises(ValueError, match="sample_list cannot pad"):
        recommend.stratified_candidates(Eu, Ei, train, [2 * n_free[0] + 1] + [10] * 9)
    ok = recommend.stratified_candidates(Eu, Ei, train, [2 * n_free[0]] + [10] * 9)
    assert len(ok[0]) == 2 * n_free[0]


def test_stratified_candidates_guards_mismatched_tables():
    eu, ei, train = _setup(3, U=8, I=300, d=64)
    Eu = torch.from_numpy(eu).to(DEV)
    with pytest.raises(TypeError):
        recommend.stratified_candidates(Eu, torch.from_numpy(ei).to(DEV).bfloat16(), train, [20] * 8)
    with pytest.raises(ValueError):
        recommend.stratified_candidates(Eu, torch.from_numpy(ei[:, :32].copy()).to(DEV), train, [20] * 8)
    mp, mi = ops.lists_to_device_csr(train, DEV)
    with pytest.raises(ValueError):
        recommend.strat_labels(Eu, torch.from_numpy(ei[:, :32].copy()).to(DEV), mp, mi, -1.0, 0.2, 10)


def test_stratified_candidates_on_a_side_stream_and_csr_input():
    """Issued under a non-default current stream (the event that guards the host read must be
    recorded where the copies run) and with the train items as a CSR pair: same lists."""
    eu, ei, train = _setup(seed=11, U=500, I=3000, d=64)
    Eu, Ei = torch.from_numpy(eu).to(DEV), torch.from_numpy(ei).to(DEV)
    targets = [200] * len(train)
    ref = recommend.stratified_candidates(Eu, Ei, train, targets, seed=4, batch=128)
    s = torch.cuda.Stream(device=DEV)
    s.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(s):
        side = recommend.stratified_candidates(Eu, Ei, train, targets, seed=4, batch=128)
    csr = ops.lists_to_device_csr(train, DEV)
    via_csr = recommend.stratified_candidates(Eu, Ei, csr, targets, seed=4, batch=128)
    assert side == ref and via_csr == ref
    assert ref == [list(r) for r in ref] and len(ref) == 500
