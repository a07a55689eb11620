"""GPU parity of SURVEY 8(f) rank 1 (candidate-level similarity) against the numpy restatements in
oracle/oracle.py (float64 products).  The reference's own code cannot be run here and
ships no fixtures for these functions: parity is against the restatement only ("parity unpinned"
beyond it).  Inputs use the reference's file formats (emb_*.npy, rating_{train,test}.csv, user.csv,
rec/<seed>/pm.npy) in a temporary data root."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle
from factors_of_serendipity_recommendation_amd import ops, recommend, serendipity

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _bf16_round(x):
    return torch.from_numpy(x).to(torch.bfloat16).float().numpy()


def _ragged(rng, n_users, n_items, lo, hi):
    return [rng.choice(n_items, size=int(rng.integers(lo, hi + 1)), replace=False).tolist() for _ in range(n_users)]


@pytest.mark.parametrize("dt,d", [(torch.float32, 8), (torch.float32, 64), (torch.float32, 100),
                                  (torch.float32, 256), (torch.bfloat16, 64), (torch.bfloat16, 256)])
@pytest.mark.parametrize("reduce", ["max", "sum"])
def test_list_dot_reduce(dt, d, reduce):
    rng = np.random.default_rng(d + (7 if reduce == "max" else 0))
    I, U = 900, 37
    T = rng.standard_normal((I, d)).astype(np.float32)
    if dt == torch.bfloat16:
        T = _bf16_round(T)
    A = _ragged(rng, U, I, 0, 100)
    B = _ragged(rng, U, I, 0, 70)
    B[3] = []  # an empty history
    got = ops.list_dot_reduce(torch.from_numpy(T).to(DEV).to(dt), ops.lists_to_device_csr(A, DEV, sort=False),
                              ops.lists_to_device_csr(B, DEV, sort=False), reduce).cpu().numpy()
    ref = np.concatenate(oracle.list_dot_reduce(T, A, B, reduce))
    assert got.shape == ref.shape
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(got), fin)
    assert np.all(got[~fin] == ref[~fin])
    scale = np.sqrt(d) * np.abs(T).max() ** 2 * (70 if reduce == "sum" else 1)
    assert np.abs(got[fin] - ref[fin]).max() <= 2e-6 * scale


@pytest.fixture
def dataset(tmp_path):
    """A small dataset directory in the reference's formats."""
    import pandas as pd
    rng = np.random.default_rng(3)
    U, I, d = 60, 500, 32
    name = "synth"
    root = tmp_path / "data"
    (root / name / "rec" / "1").mkdir(parents=True)
    eu = (rng.standard_normal((U, d)) * 0.3).astype(np.float32)
    ei = (rng.standard_normal((I, d)) * 0.3).astype(np.float32)
    np.save(root / name / "emb_user.npy", eu)
    np.save(root / name / "emb_item.npy", ei)
    train = _ragged(rng, U, I, 3, 40)
    test = _ragged(rng, U, I, 1, 10)
    for fname, lists in (("rating_train.csv", train), ("rating_test.csv", test)):
        rows = [(u, i) for u, l in enumerate(lists) for i in l]
        pd.DataFrame(rows, columns=["userInd", "itemInd"]).to_csv(root / name / fname, index=False)
    num_item = np.array([len(l) for l in train])
    pd.DataFrame({"userInd": np.arange(U), "num_item": num_item}).to_csv(root / name / "user.csv", index=False)
    cands = {u: rng.choice(I, 200, replace=False).tolist() for u in range(U)}
    pm = np.stack([rng.choice(cands[u], 20, replace=False) for u in range(U)])
    np.save(root / name / "rec" / "1" / "pm.npy", pm)
    return dict(root=str(root), name=name, eu=eu, ei=ei, train=train, test=test, num_item=num_item,
                cands=cands, pm=pm)


def _same_sets_modulo_ties(got, ref, key_fn):
    for u in range(got.shape[0]):
        g, r = set(got[u].tolist()), set(ref[u].tolist())
        if g == r:
            continue
        keys = key_fn(u)
        kth = min(keys[x] for x in r)
        for x in g ^ r:
            assert abs(keys[x] - kth) < 1e-5, (u, x)


def test_item_dot_minmax(dataset):
    mn, mx = recommend.item_dot_minmax(torch.from_numpy(dataset["ei"]).to(DEV))
    rmn, rmx = oracle.item_dot_minmax(dataset["ei"])
    assert abs(mn - rmn) < 1e-5 and abs(mx - rmx) < 1e-5


def test_difference_dropin(dataset):
    ds = dataset
    recommend.difference(ds["cands"], ds["name"], 1, K=20, data_root=ds["root"], device=DEV)
    got = np.load(os.path.join(ds["root"], ds["name"], "rec", "1", "rec_dif.npy"))
    ref = oracle.difference(ds["ei"], ds["cands"], ds["train"], K=20)
    assert got.shape == ref.shape == (60, 20)
    mn, mx = oracle.item_dot_minmax(ds["ei"])
    E = ds["ei"].astype(np.float64)

    def key(u):
        m = (E @ E[ds["train"][u]].T).max(axis=1)
        return 1 - (m - mn) / (mx - mn)
    _same_sets_modulo_ties(got, ref, key)


def test_elasticity_dropin(dataset):
    ds = dataset
    recommend.elasticity_item(ds["cands"], ds["name"], 1, K=20, alpha=1.0, data_root=ds["root"], device=DEV)
    got = np.load(os.path.join(ds["root"], ds["name"], "rec", "1", "rec_ela.npy"))
    ref = oracle.elasticity_item(ds["eu"], ds["ei"], ds["cands"], ds["num_item"], K=20, alpha=1.0)
    assert got.shape == ref.shape
    assert np.mean([len(set(a) & set(b)) / 20 for a, b in zip(got.tolist(), ref.tolist())]) > 0.99


def test_ser1_ser2_diversity(dataset):
    ds = dataset
    mn, mx = oracle.item_dot_minmax(ds["ei"])
    mat_rec = np.stack([np.asarray(ds["cands"][u][:20]) for u in range(60)])
    got = serendipity.ser1(ds["name"], mat_rec, mx, mn, data_root=ds["root"], device=DEV)
    ref = oracle.ser1(ds["ei"], mat_rec, ds["train"], ds["test"], mx, mn)
    for g, r in zip(got[:3], ref[:3]):
        assert abs(g - r) < 1e-5
    assert np.allclose(got[3], ref[3], atol=1e-5) and np.allclose(got[4], ref[4], atol=1e-5)
    g2 = serendipity.ser2(ds["name"], mat_rec, mx, mn, 1, data_root=ds["root"], device=DEV)
    r2 = oracle.ser2(ds["ei"], mat_rec, ds["pm"], ds["train"], mx, mn)
    assert abs(g2 - r2) < 1e-5
    gd = serendipity.diversity(ds["name"], mat_rec, mx, mn, data_root=ds["root"], device=DEV)
    rd = oracle.diversity(ds["ei"], mat_rec, mx, mn)
    assert abs(gd - rd) < 1e-5
