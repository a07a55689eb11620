"""GPU: the drop-ins fail where the reference fails, and caches see every parameter update.

  * eval -> train step -> eval: LightGCN's eval-mode propagation cache must not serve tables from
    before the step (train.Adam writes the weights through a raw pointer; model.py:145-184 recomputes
    computer() on every getUsersRating call, so the reference never returns stale tables);
  * gather_scores: candidate ids outside the item table raise IndexError (numpy indexing in
    recommend.py:167-171, :214-217), and fewer candidate lists than user rows is legal;
  * ragged_topk: a list shorter than K raises (np.argpartition(score, -K), recommend.py:53-56);
  * bpr_loss: an out-of-range user / item id raises IndexError (torch indexing, model.py:186-195).
"""
import numpy as np
import pytest
import torch

from factors_of_serendipity_recommendation_amd import ops, recommend, train

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _loader(mlls, tmp_path):
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


def _model(ds):
    from factors_of_serendipity_recommendation_amd.model import LightGCN
    torch.manual_seed(0)
    cfg = {"latent_dim_rec": 64, "lightGCN_n_layers": 3, "keep_prob": 0.6, "A_split": False, "pretrain": 0,
           "dropout": 0, "decay": 1e-4, "lr": 0.01}
    return LightGCN(cfg, ds).to(DEV), cfg


def test_eval_cache_sees_the_optimizer_step(mlls, tmp_path):
    ds = _loader(mlls, tmp_path)
    model, cfg = _model(ds)
    bpr = train.BPRLoss(model, cfg)
    users = torch.arange(16, device=DEV)
    model.eval()
    with torch.no_grad():
        r0 = model.getUsersRating(users).clone()
        r0b = model.getUsersRating(users)
    assert torch.equal(r0, r0b)  # the cache serves an unchanged model
    model.train()
    u = torch.randint(0, ds.n_users, (512,), device=DEV)
    p = torch.randint(0, ds.m_items, (512,), device=DEV)
    n = torch.randint(0, ds.m_items, (512,), device=DEV)
    bpr.stageOne(u, p, n)
    model.eval()
    with torch.no_grad():
        r1 = model.getUsersRating(users)
        u2, i2 = model.computer()
        fresh = torch.sigmoid(u2[:16] @ i2.T)
    assert not torch.equal(r0, r1), "eval after a train step returned the pre-step ratings"
    assert torch.allclose(r1, fresh, rtol=1e-5, atol=1e-6)


def test_train_epoch_then_eval_is_fresh(mlls, tmp_path):
    from factors_of_serendipity_recommendation_amd import evaluator, sampling
    ds = _loader(mlls, tmp_path)
    model, cfg = _model(ds)
    bpr = train.BPRLoss(model, cfg)
    model.eval()
    with torch.no_grad():
        before = model.getUsersRating(torch.arange(8, device=DEV)).clone()
    res0 = evaluator.Test(ds, model, topks=[20])
    sampling.seed(7)
    train.BPR_train_original(ds, model, bpr, 0, batch_size=2048, device=DEV)
    model.eval()
    with torch.no_grad():
        after = model.getUsersRating(torch.arange(8, device=DEV))
    assert not torch.equal(before, after)
    res1 = evaluator.Test(ds, model, topks=[20])
    assert res0["recall"][0] != res1["recall"][0] or res0["ndcg"][0] != res1["ndcg"][0]


def test_gather_scores_fewer_lists_than_users_and_bad_ids():
    rng = np.random.default_rng(3)
    U, I, d = 50, 300, 64
    eu = torch.from_numpy(rng.standard_normal((U, d)).astype(np.float32)).to(DEV)
    ei = torch.from_numpy(rng.standard_normal((I, d)).astype(np.float32)).to(DEV)
    lists = [rng.choice(I, 30, replace=False).tolist() for _ in range(10)]  # 10 lists, 50 user rows
    scores, indptr, items = recommend.candidate_scores(eu, ei, lists)
    ref = np.concatenate([eu[j].cpu().numpy() @ ei[lists[j]].cpu().numpy().T for j in range(10)])
    assert scores.numel() == 300
    assert np.allclose(scores.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    with pytest.raises(IndexError):
        recommend.candidate_scores(eu, ei, [[0, 1, I]])
    with pytest.raises(IndexError):
        recommend.candidate_scores(eu, ei, [[-1, 2]])
    with pytest.raises(ValueError):
        recommend.candidate_scores(eu[:2], ei, [[0], [1], [2]])  # 3 lists, 2 user rows


def test_ragged_topk_short_list_raises():
    rng = np.random.default_rng(4)
    eu = torch.from_numpy(rng.standard_normal((3, 16)).astype(np.float32)).to(DEV)
    ei = torch.from_numpy(rng.standard_normal((100, 16)).astype(np.float32)).to(DEV)
    with pytest.raises(ValueError):
        recommend.topk_candidates(eu, ei, [list(range(30)), list(range(5)), list(range(40))], K=20)
    got = recommend.topk_candidates(eu, ei, [list(range(30)), list(range(20)), list(range(40))], K=20)
    assert sorted(got[1].tolist()) == list(range(20))


def test_bpr_loss_bad_index_raises(mlls, tmp_path):
    ds = _loader(mlls, tmp_path)
    model, _ = _model(ds)
    u = torch.tensor([0, 1], device=DEV)
    ok = torch.tensor([2, 3], device=DEV)
    loss, reg = model.bpr_loss(u, ok, ok)
    assert torch.isfinite(loss) and torch.isfinite(reg)
    with pytest.raises(IndexError):
        model.bpr_loss(u, torch.tensor([2, ds.m_items], device=DEV), ok)
    with pytest.raises(IndexError):
        model.bpr_loss(torch.tensor([0, ds.n_users], device=DEV), ok, ok)
    with pytest.raises(IndexError):
        model.bpr_loss(u, ok, torch.tensor([-1, 3], device=DEV))
