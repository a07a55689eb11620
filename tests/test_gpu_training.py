"""GPU: BPR sampling (sources/sampling.cpp:27-86) and the BPR training epoch
(Procedure.BPR_train_original, code/Procedure.py:26-57) through the HIP propagation.

The reference sampler draws from libc rand() seeded by the clock, so parity is distributional:
row layout, every positive is a positive, no negative is, negatives uniform over the non-positives
(chi-square), determinism per seed (parity unpinned beyond these properties)."""
import numpy as np
import pytest
import torch

from factors_of_serendipity_recommendation_amd import ops, sampling, train

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _pos_lists(rng, U, I):
    return [np.sort(rng.choice(I, size=int(rng.integers(0, 40)), replace=False)).tolist() for _ in range(U)]


def test_sampler_rows_are_valid_and_deterministic():
    rng = np.random.default_rng(1)
    U, I = 300, 700
    allPos = _pos_lists(rng, U, I)
    allPos[5] = []  # no positives: no rows
    pos = ops.lists_to_device_csr(allPos, DEV)
    S = sampling.sample_device(pos, I, per_user=7, neg_num=3, seed_value=11).cpu().numpy()
    S2 = sampling.sample_device(pos, I, per_user=7, neg_num=3, seed_value=11).cpu().numpy()
    S3 = sampling.sample_device(pos, I, per_user=7, neg_num=3, seed_value=12).cpu().numpy()
    assert np.array_equal(S, S2) and not np.array_equal(S, S3)
    assert S.shape[1] == 5
    n_with = sum(1 for p in allPos if p)
    assert S.shape[0] == 7 * n_with
    counts = np.bincount(S[:, 0], minlength=U)
    assert all(counts[u] == (7 if allPos[u] else 0) for u in range(U))
    for row in S:
        p = set(allPos[row[0]])
        assert row[1] in p
        assert all(0 <= x < I and x not in p for x in row[2:])


def test_sampler_by_user_and_uniform_negatives():
    rng = np.random.default_rng(2)
    I = 400
    allPos = [np.sort(rng.choice(I, 60, replace=False)).tolist(), [3, 9]]
    users = np.zeros(200_000, dtype=np.int32)
    S = sampling.sample_negative_ByUser(users, I, allPos, 1)
    assert S.shape == (200_000, 3) and (S[:, 0] == 0).all()
    pos = set(allPos[0])
    assert not np.isin(S[:, 2], list(pos)).any()
    c = np.bincount(S[:, 2], minlength=I)[[i for i in range(I) if i not in pos]]
    expected = len(users) / len(c)
    chi2 = ((c - expected) ** 2 / expected).sum()
    dof = len(c) - 1
    assert chi2 < dof + 6 * np.sqrt(2 * dof), chi2  # ~6 sigma
    pc = np.bincount(S[:, 1], minlength=I)[allPos[0]]
    assert pc.min() > 0.7 * len(users) / 60 and pc.max() < 1.3 * len(users) / 60


def test_bpr_epoch_through_hip_propagation(mlls, tmp_path):
    from factors_of_serendipity_recommendation_amd.dataloader import Loader
    from factors_of_serendipity_recommendation_amd.model import LightGCN
    tp, tx = mlls["train_list_indptr"], mlls["train_list_indices"]
    with open(tmp_path / "train.txt", "w") as f:
        for j, u in enumerate(mlls["train_list_users"]):
            f.write(" ".join(str(x) for x in [u] + list(tx[tp[j]:tp[j + 1]])) + "\n")
    sp_, sx = mlls["test_indptr"], mlls["test_indices"]
    with open(tmp_path / "test.txt", "w") as f:
        for j, u in enumerate(mlls["test_users"]):
            f.write(" ".join(str(x) for x in [u] + list(sx[sp_[j]:sp_[j + 1]])) + "\n")
    ds = Loader(path=str(tmp_path), device=DEV)
    torch.manual_seed(0)
    cfg = {"latent_dim_rec": 64, "lightGCN_n_layers": 3, "keep_prob": 0.6, "A_split": False, "pretrain": 0,
           "dropout": 0, "decay": 1e-4, "lr": 0.001}
    model = LightGCN(cfg, ds).to(DEV)
    bpr = train.BPRLoss(model, cfg)
    sampling.seed(2020)
    losses = []
    for epoch in range(3):
        msg = train.BPR_train_original(ds, model, bpr, epoch, batch_size=2048, device=DEV)
        assert msg.startswith("loss")
        losses.append(float(msg[4:msg.index("-")]))
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses


def test_captured_epoch_equals_eager_epoch(mlls, tmp_path):
    """BPR_train_original with the minibatch captured as a hipGraph (the default) against the eager
    loop, from the same weights and sampler seed: the same parameters after two epochs (to the
    f32 atomics' summation-order noise of the fused loss backward), the same Adam step count, and
    the eval-mode propagation cache sees the replayed updates."""
    from factors_of_serendipity_recommendation_amd.dataloader import Loader
    from factors_of_serendipity_recommendation_amd.model import LightGCN
    tp, tx = mlls["train_list_indptr"], mlls["train_list_indices"]
    with open(tmp_path / "train.txt", "w") as f:
        for j, u in enumerate(mlls["train_list_users"]):
            f.write(" ".join(str(x) for x in [u] + list(tx[tp[j]:tp[j + 1]])) + "\n")
    with open(tmp_path / "test.txt", "w") as f:
        f.write(f"{int(mlls['train_list_users'][0])} {int(tx[0])}\n")
    ds = Loader(path=str(tmp_path), device=DEV)
    cfg = {"latent_dim_rec": 64, "lightGCN_n_layers": 3, "keep_prob": 0.6, "A_split": False, "pretrain": 0,
           "dropout": 0, "decay": 1e-4, "lr": 0.001}
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        model = LightGCN(cfg, ds).to(DEV)
        bpr = train.BPRLoss(model, cfg)
        model.eval()
        with torch.no_grad():
            before = model.getUsersRating(torch.arange(4, device=DEV)).clone()
        sampling.seed(7)
        for epoch in range(2):
            train.BPR_train_original(ds, model, bpr, epoch, batch_size=512, device=DEV, graph=graph)
        model.eval()
        with torch.no_grad():
            after = model.getUsersRating(torch.arange(4, device=DEV))
        assert not torch.equal(before, after), "eval cache kept the pre-training propagation"
        steps = [float(st["step"]) for st in bpr.opt.state.values()]
        runs.append(([p.detach().clone() for p in model.parameters()], steps))
    (pe, se), (pg, sg) = runs
    rows = ds.n_users * max(1, ds.trainDataSize // ds.n_users)  # the epoch's sample rows (train.py)
    n_batches = 2 * (-(-rows // 512))
    assert se == sg and all(x == n_batches for x in sg), (se, sg, n_batches)
    for a, b in zip(pe, pg):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5 * b.abs().max().item())


def test_captured_step_recaptures_on_lr_change_and_state_reload(mlls, tmp_path):
    """The captured minibatch freezes lr / betas / eps / decay and the optimizer state addresses:
    a scheduler-style lr change between epochs and an opt.load_state_dict (new state tensors) must
    re-capture, so the captured run still equals the eager run with the same changes."""
    import copy
    from factors_of_serendipity_recommendation_amd.dataloader import Loader
    from factors_of_serendipity_recommendation_amd.model import LightGCN
    tp, tx = mlls["train_list_indptr"], mlls["train_list_indices"]
    with open(tmp_path / "train.txt", "w") as f:
        for j, u in enumerate(mlls["train_list_users"]):
            f.write(" ".join(str(x) for x in [u] + list(tx[tp[j]:tp[j + 1]])) + "\n")
    with open(tmp_path / "test.txt", "w") as f:
        f.write(f"{int(mlls['train_list_users'][0])} {int(tx[0])}\n")
    ds = Loader(path=str(tmp_path), device=DEV)
    cfg = {"latent_dim_rec": 64, "lightGCN_n_layers": 3, "keep_prob": 0.6, "A_split": False, "pretrain": 0,
           "dropout": 0, "decay": 1e-4, "lr": 0.001}
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        model = LightGCN(cfg, ds).to(DEV)
        bpr = train.BPRLoss(model, cfg)
        sampling.seed(11)
        train.BPR_train_original(ds, model, bpr, 0, batch_size=512, device=DEV, graph=graph)
        for g in bpr.opt.param_groups:
            g["lr"] = 0.01  # a scheduler step
        train.BPR_train_original(ds, model, bpr, 1, batch_size=512, device=DEV, graph=graph)
        bpr.opt.load_state_dict(copy.deepcopy(bpr.opt.state_dict()))  # new state tensors
        train.BPR_train_original(ds, model, bpr, 2, batch_size=512, device=DEV, graph=graph)
        if graph:
            assert bpr._lgx_captured.captures == 3
        runs.append([p.detach().clone() for p in model.parameters()])
    for a, b in zip(*runs):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5 * b.abs().max().item())


# ---------------------------------------------------------------- fused BPR loss (csrc/bpr.hip)
def _torch_bpr(light, wu, wi, users, pos, neg):
    """model.py:196-209 in the reference's torch ops (fp32), the parity reference."""
    U = wu.shape[0]
    ue, pe, ne = light[users], light[U + pos], light[U + neg]
    reg = 0.5 * (wu[users].norm(2).pow(2) + wi[pos].norm(2).pow(2) + wi[neg].norm(2).pow(2)) / float(len(users))
    loss = torch.mean(torch.nn.functional.softplus(torch.sum(ue * ne, 1) - torch.sum(ue * pe, 1)))
    return loss, reg


@pytest.mark.parametrize("d,B", [(64, 2048), (64, 37), (30, 500), (128, 4096)])
def test_fused_bpr_loss_matches_torch(d, B):
    """Loss, reg and all three gradients vs the torch-op formulation in fp32 (rel 1e-5 on the
    scalars, 1e-5 of the gradient scale elementwise); duplicated users / items exercise the
    scatter accumulation; grad_loss / grad_reg != 1 exercise the upstream scaling."""
    from factors_of_serendipity_recommendation_amd.model import _BPRLoss
    g = torch.Generator().manual_seed(d * 1000 + B)
    U, I = 300, 500
    light = (torch.randn(U + I, d, generator=g) * 0.5).to(DEV)
    wu = (torch.randn(U, d, generator=g) * 0.1).to(DEV)
    wi = (torch.randn(I, d, generator=g) * 0.1).to(DEV)
    users = torch.randint(0, U, (B,), generator=g).to(DEV)
    pos = torch.randint(0, I, (B,), generator=g).to(DEV)
    neg = torch.randint(0, I, (B,), generator=g).to(DEV)
    ins = [t.clone().requires_grad_(True) for t in (light, wu, wi)]
    ref = [t.clone().requires_grad_(True) for t in (light, wu, wi)]
    loss, reg = _BPRLoss.apply(*ins, users, pos, neg)
    rl, rr = _torch_bpr(*ref, users, pos, neg)
    assert torch.allclose(loss, rl, rtol=1e-5, atol=0) and torch.allclose(reg, rr, rtol=1e-5, atol=0), \
        (loss.item(), rl.item(), reg.item(), rr.item())
    (0.7 * loss + 3e-2 * reg).backward()
    (0.7 * rl + 3e-2 * rr).backward()
    for a, b in zip(ins, ref):
        scale = b.grad.abs().max().item()
        assert (a.grad - b.grad).abs().max().item() <= 1e-5 * scale + 1e-9


def test_fused_bpr_loss_flags_bad_index():
    U, I, d = 10, 20, 64
    light = torch.zeros(U + I, d, device=DEV)
    wu, wi = torch.zeros(U, d, device=DEV), torch.zeros(I, d, device=DEV)
    idx = torch.tensor([0, 1, 2], device=DEV)
    loss, reg, _ = ops.bpr_loss_forward(light, wu, wi, idx, idx, torch.tensor([0, I, 2], device=DEV))
    assert torch.isnan(loss).item()
    loss, reg, _ = ops.bpr_loss_forward(light, wu, wi, idx, idx, idx)
    assert abs(loss.item() - np.log(2.0)) < 1e-7 and reg.item() == 0.0


def test_model_bpr_loss_fused_equals_reference_form(mlls):
    """LightGCN.bpr_loss (fused) against bpr_loss_torch (the reference's ops) on the mlls graph:
    same loss, and the same embedding-weight gradients after backward through the propagation."""
    from factors_of_serendipity_recommendation_amd import build_norm_adj
    from factors_of_serendipity_recommendation_amd.model import LightGCN

    class _DS:
        pass

    U, I = int(mlls["n_users"]), int(mlls["n_items"])
    ds = _DS()
    ds.n_users, ds.m_items = U, I
    A = build_norm_adj(mlls["train_users"], mlls["train_items"], U, I, dedup=True, device=DEV)
    ds.getSparseGraph = lambda: None
    ds.getCSRGraph = lambda: A
    torch.manual_seed(3)
    cfg = {"latent_dim_rec": 64, "lightGCN_n_layers": 3, "pretrain": 0, "dropout": 0}
    model = LightGCN(cfg, ds).to(DEV)
    gen = torch.Generator().manual_seed(5)
    users = torch.randint(0, U, (2048,), generator=gen).to(DEV)
    pos = torch.randint(0, I, (2048,), generator=gen).to(DEV)
    neg = torch.randint(0, I, (2048,), generator=gen).to(DEV)
    grads = []
    for fn in (model.bpr_loss, model.bpr_loss_torch):
        model.zero_grad()
        loss, reg = fn(users, pos, neg)
        (loss + 1e-4 * reg).backward()
        grads.append((loss.item(), reg.item(), model.embedding_user.weight.grad.clone(),
                      model.embedding_item.weight.grad.clone()))
    (l1, r1, gu1, gi1), (l2, r2, gu2, gi2) = grads
    assert abs(l1 - l2) <= 1e-5 * abs(l2) and abs(r1 - r2) <= 1e-5 * abs(r2)
    for a, b in ((gu1, gu2), (gi1, gi2)):
        assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item()


@pytest.mark.parametrize("n", [4 * 70_839 * 16, 1001])
def test_lgx_adam_matches_torch_adam(n):
    """train.Adam (one lgx_adam_step pass) against torch.optim.Adam(lr) over 6 steps: parameters and
    both moments within fp32 rounding (1e-6 relative, 1e-6 of the tensor's scale absolute -- a
    moment near a zero crossing keeps the rounding of its inputs), the updates to 1e-4 relative;
    an odd length exercises the tail."""
    from factors_of_serendipity_recommendation_amd import train
    g = torch.Generator().manual_seed(n)
    p0 = torch.randn(n, generator=g).to(DEV)
    grads = [torch.randn(n, generator=g).to(DEV) * s for s in (1.0, 0.1, 0.0, 3.0, 1e-3, 1.0)]
    a = torch.nn.Parameter(p0.clone())
    b = torch.nn.Parameter(p0.clone())
    oa, ob = train.Adam([a], lr=1e-3), torch.optim.Adam([b], lr=1e-3)
    for gr in grads:
        a.grad, b.grad = gr.clone(), gr.clone()
        oa.step()
        ob.step()
    for x, y in ((a, b), (oa.state[a]["exp_avg"], ob.state[b]["exp_avg"]),
                 (oa.state[a]["exp_avg_sq"], ob.state[b]["exp_avg_sq"])):
        x, y = x.detach(), y.detach()
        assert torch.allclose(x, y, rtol=1e-6, atol=1e-6 * y.abs().max().item())
    # the parameter updates themselves (~6e-3): equal to 1e-4 relative, plus the few ulps of |p|
    # that 6 roundings of p itself leave (1e-6 |p| = 8 ulps)
    da, db = a.detach() - p0, b.detach() - p0
    assert ((da - db).abs() <= 1e-4 * db.abs() + 1e-6 * p0.abs() + 1e-9).all()
    assert float(oa.state[a]["step"]) == 6.0
