"""GPU: the evaluator's two-route split pinned at the shapes its a7 / a8 rows are timed on.

Procedure.Test (lightGCN/LightGCN-PyTorch-master/code/Procedure.py:121-146) and TF batch_test
(LightGCN-tf/utility/batch_test.py:41-65) rank every test user's items with its train items masked.
evaluator._Route sends users whose mask is longer than dense_mask_min(...) to dense score rows on a
side stream (ops.score_topk_dense_masked: score_dense -> -inf scatter -> topk_rows) and the rest to
the fused score + mask + top-k launch.  Here both routes run at the synthetic Gowalla shape (27 522
test users x 40 981 items, d = 64, ~1 200 dense-route users) and the Amazon-book shape (52 643 x
91 599, d = 128, ~4 900 dense-route users, the dense route forced into 3 chunks), on propagated
LightGCN tables, with each user's train items as the mask -- the tables the rows are timed on.

Every dense-route user and 2 000 fused-route users spread over all workgroups are checked against
float64 scores of the same f32 tables: 20 distinct unmasked items, each scoring at least the exact
k-th best unmasked score minus the near-tie tolerance.  Both kernels rank raw f32 dot products (the
fused launch applies its sigmoid only to the values it returns), so two items whose float64 scores
are closer than the f32 rounding of a dot product can come out in either order: the tolerance is
twice the f32 dot-product error bound, 2 * d * 2^-24 * |q_u| * max_i |e_i| (DESIGN.md §4, round 5:
one Amazon-book user of 52 643 flipped by 1.2e-7).  How many users' sets differ from the float64
sets at all is asserted small as well.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _eval_dataset(cfg, tmpdir):
    """The config's synthetic graph in the reference's txt format: every 5th edge of a user (sorted by
    item) is a test interaction, the rest train (users with < 2 edges: train only) -- the datasets
    tools/bench_rows.py times the a7 / a8 rows on."""
    from factors_of_serendipity_recommendation_amd.dataloader import Loader
    from factors_of_serendipity_recommendation_amd.synth import synth_edges
    u, i = synth_edges(cfg, 2020, DEV)
    u, i = u.cpu().numpy(), i.cpu().numpy()
    order = np.lexsort((i, u))
    u, i = u[order], i[order]
    bounds = np.searchsorted(u, np.arange(cfg.n_users + 1))
    pos = np.arange(len(u)) - bounds[u]
    deg = np.diff(bounds)[u]
    test = (pos % 5 == 4) & (deg >= 2)
    path = os.path.join(tmpdir, f"eval_{cfg.name}")
    os.makedirs(path, exist_ok=True)
    for name, sel in (("train.txt", ~test), ("test.txt", test)):
        uu, ii = u[sel], i[sel]
        b = np.searchsorted(uu, np.arange(cfg.n_users + 1))
        with open(os.path.join(path, name), "w") as f:
            for x in range(cfg.n_users):
                if b[x + 1] > b[x]:
                    f.write(str(x) + " " + " ".join(map(str, ii[b[x]:b[x + 1]])) + "\n")
    return Loader(path=path, device=DEV, cache_adj=False)


def _check_against_float64(U, I, rows, mask, idx, positions, k):
    """(number of users whose set differs from the float64 top-k set, worst margin / tolerance)."""
    ip, ix = mask[0].cpu().numpy(), mask[1].cpu().numpy()
    Id = I.double()
    imax = float(I.double().norm(dim=1).max())
    d = I.shape[1]
    differ, worst = 0, 0.0
    for c0 in range(0, len(positions), 1024):
        pos = positions[c0:c0 + 1024]
        q = U[rows[pos]].double()
        S = q @ Id.T
        for j, p in enumerate(pos.tolist()):
            m = torch.from_numpy(ix[ip[p]:ip[p + 1]].astype(np.int64)).to(DEV)
            S[j, m] = float("-inf")
        got_idx = idx[pos].long()
        assert (got_idx >= 0).all()
        srt = got_idx.sort(1).values
        assert (srt[:, 1:] != srt[:, :-1]).all(), "an item repeats in a list"
        got = S.gather(1, got_idx)
        assert torch.isfinite(got).all(), "a masked item was returned"
        top = torch.topk(S, k, dim=1)
        kth = top.values[:, -1:]
        tol = 2 * d * 2.0 ** -24 * q.norm(dim=1, keepdim=True) * imax
        short = (kth - got) / tol
        worst = max(worst, float(short.max()))
        assert (got >= kth - tol).all(), f"an item below the k-th score by more than the tolerance ({worst:.2f})"
        ref_set = top.indices.sort(1).values
        differ += int((ref_set != srt).any(1).sum())
    return differ, worst


@pytest.mark.parametrize("name,min_heavy,chunks", [("gowalla", 1000, 1), ("amazon", 4000, 3)])
def test_two_route_evaluator_at_the_timed_shapes(tmp_path, name, min_heavy, chunks):
    from factors_of_serendipity_recommendation_amd import evaluator, ops
    from factors_of_serendipity_recommendation_amd.model import LightGCN
    from factors_of_serendipity_recommendation_amd.synth import CONFIGS
    cfg = CONFIGS[name]
    ds = _eval_dataset(cfg, str(tmp_path))
    conf = {"latent_dim_rec": cfg.d, "lightGCN_n_layers": cfg.K, "keep_prob": 0.6, "A_split": False,
            "pretrain": 0, "dropout": 0}
    torch.manual_seed(0)
    model = LightGCN(conf, ds).to(DEV).eval()
    with torch.no_grad():
        U, I = model.computer()
    n_items, k = I.shape[0], 20
    tl = evaluator._TestLists.get(ds, n_items, U.device)
    rule = tl.route(n_items, k, cfg.d)  # the route evaluator.Test takes
    assert rule.n_heavy >= min_heavy, rule.n_heavy
    if chunks > 1:  # the same split with the dense route in `chunks` score chunks
        step = -(-rule.n_heavy // chunks)
        r = evaluator._Route(tl.rows, tl.mask, n_items, k, cfg.d, chunk_bytes=step * n_items * 4)
        assert len(r.heavy_offsets) == chunks and r.n_heavy == rule.n_heavy
    else:
        r = rule
    idx = r.topk(U, I, k, -float(1 << 10), True)  # Procedure.Test's mask value and sigmoid
    torch.cuda.synchronize()
    # batch_test's form (raw scores, -inf mask) through the same route: the same lists
    idx_bt = r.topk(U, I, k, float("-inf"), False)
    assert torch.equal(idx, idx_bt)
    light = r.light_pos
    sample = light[torch.linspace(0, light.numel() - 1, 2000, device=DEV).round().long()]
    positions = torch.cat([r.heavy_pos, sample])
    differ, worst = _check_against_float64(U, I, tl.rows, tl.mask, idx, positions, k)
    # near-tie flips are rare: at most 1 % of the checked users' sets differ from float64's
    assert differ <= positions.numel() // 100, (differ, positions.numel(), worst)
    print(f"{name}: {r.n_heavy} dense-route users in {len(r.heavy_offsets)} chunk(s), {positions.numel()} "
          f"users checked, {differ} sets differ from float64 within the tolerance (worst {worst:.3f} of it)")
    # evaluator.Test's metrics are those of these lists
    got = evaluator.Test(ds, model, topks=[k])
    sums = ops.test_metrics(idx, tl.truth, [k], tl.recall_n_dev).cpu().numpy()
    assert np.allclose(got["recall"], sums[0] / len(tl.users), rtol=1e-12, atol=0)


def test_batch_test_and_procedure_test_at_the_gowalla_shape_vs_oracle(tmp_path):
    """evaluator.batch_test (TF batch_test.py:25-84, train items masked with -inf) and evaluator.Test
    (Procedure.py:96-174) at the synthetic Gowalla shape, where ~1 250 users take the dense route,
    against the oracle's restatements on the same propagated f32 tables: oracle.batch_test (float64
    dots rounded to f32, per 1024-user batch) and Procedure.Test's metrics over the oracle's own
    float64 top-20 lists.  The two sides rank f32 scores summed in different orders, so a near-tie may
    swap (the lists test above: none at this shape); the metric means may then move by one user's
    share: atol 1e-4."""
    from oracle import oracle
    from factors_of_serendipity_recommendation_amd import evaluator
    from factors_of_serendipity_recommendation_amd.model import LightGCN
    from factors_of_serendipity_recommendation_amd.synth import CONFIGS
    cfg = CONFIGS["gowalla"]
    ds = _eval_dataset(cfg, str(tmp_path))
    conf = {"latent_dim_rec": cfg.d, "lightGCN_n_layers": cfg.K, "keep_prob": 0.6, "A_split": False,
            "pretrain": 0, "dropout": 0}
    torch.manual_seed(0)
    model = LightGCN(conf, ds).to(DEV).eval()
    with torch.no_grad():
        U, I = model.computer()
    users = [int(u) for u in ds.testDict.keys()]
    train = {u: [int(x) for x in p] for u, p in zip(users, ds.getUserPosItems(users))}
    test = {u: [int(x) for x in ds.testDict[u]] for u in users}
    r = evaluator._BatchLists.get(users, train, test, 0, U.device).route(I.shape[0], 20, cfg.d)
    assert r.n_heavy >= 1000, r.n_heavy
    got = evaluator.batch_test(U, I, users, train, test, Ks=[20, 10], train_set_flag=0)
    Un, In = U.cpu().numpy(), I.cpu().numpy()
    ref = oracle.batch_test(Un, In, users, train, test, Ks=[20, 10], train_set_flag=0)
    for key in ("precision", "recall", "ndcg"):
        assert np.allclose(got[key], ref[key], rtol=0, atol=1e-4), (key, got[key], ref[key])
    # Procedure.Test: sigmoid scores, train items at -(1 << 10), top-20, torch-style sums
    gt = evaluator.Test(ds, model, topks=[20])
    oidx = []
    for u0 in range(0, len(users), 2048):
        ub = users[u0:u0 + 2048]
        S = Un[ub].astype(np.float64) @ In.astype(np.float64).T
        for j, u in enumerate(ub):
            S[j, train[u]] = -np.inf
        part = np.argpartition(-S, 20, axis=1)[:, :20]
        order = np.argsort(-np.take_along_axis(S, part, 1), axis=1, kind="stable")
        oidx.append(np.take_along_axis(part, order, 1))
    want = oracle.torch_style_metrics(np.concatenate(oidx), [test[u] for u in users], [20])
    for key in ("recall", "precision", "ndcg"):
        assert np.allclose(gt[key], want[key] / len(users), rtol=0, atol=1e-4), (key, gt[key], want[key])
