"""GPU: the fp32 scoring path (the reference's precision: model.py:183 fp32 matmul + Procedure.py:
134-135 mask and torch.topk) through score_topk_f32_lds -- the LDS-ring walk on
v_mfma_f32_16x16x4_f32, 4 waves x 32 users (d > 128) or 8 staggered waves x 32 users (d <= 128) --
in every launch mode the planner uses: catalog split (small batches), full sweep (>= 256 user
tiles), full sweep seeded in stages (>= 262 144 items), the split tail
of a partial last round, user_rows, the min / max variant; and the fall-back kernel where the LDS
budget rules the walk out (d = 256 with k > 20).  Checked on the device against float64 scores:
k distinct unmasked items, each within 1e-5 of the exact k-th best, values = the float64 scores to
1e-5 (fp32 products and sums of |x| ~ 1 inputs over d <= 256)."""
import numpy as np
import pytest
import torch

import factors_of_serendipity_recommendation_amd as lgx
from factors_of_serendipity_recommendation_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _mask(B, I, per, g):
    m = torch.randint(0, I, (B, per), device=DEV, generator=g).sort(1).values
    keep = torch.ones_like(m, dtype=torch.bool)
    keep[:, 1:] = m[:, 1:] != m[:, :-1]
    indptr = torch.zeros(B + 1, dtype=torch.int64, device=DEV)
    indptr[1:] = torch.cumsum(keep.sum(1), 0)
    return indptr, m[keep].to(torch.int32)


def _check(Q, items, idx, val, mask, sel, k, user_rows=None, chunk=250):
    items64 = items.double()
    for c0 in range(0, sel.numel(), chunk):
        s = sel[c0:c0 + chunk]
        qs = user_rows[s] if user_rows is not None else s
        S = Q[qs].double() @ items64.T
        if mask is not None:
            indptr, mi = mask
            for j, u in enumerate(s.tolist()):
                S[j, mi[indptr[u]:indptr[u + 1]].long()] = float("-inf")
        kth = torch.topk(S, k, dim=1).values[:, -1:]
        got_idx = idx[s].long()
        assert (got_idx >= 0).all()
        got = S.gather(1, got_idx)
        assert torch.isfinite(got).all(), "a masked item was returned"
        assert (got >= kth - 1e-5 * kth.abs().clamp(min=1.0)).all()
        srt = got_idx.sort(1).values
        assert (srt[:, 1:] != srt[:, :-1]).all()
        assert torch.allclose(val[s].double(), got, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("d,k,lds,waves", [(64, 20, True, 8), (128, 20, True, 8), (128, 32, True, 4),
                                           (192, 7, True, 4), (256, 20, True, 4), (256, 21, False, 0),
                                           (96, 20, False, 0), (32, 20, False, 0)])
def test_f32_kernel_selection(d, k, lds, waves):
    plan = ops.score_topk_plan(65_536, 100_000, d, torch.float32, k)
    assert plan.startswith("score_topk_f32_lds") == lds, plan
    if lds:
        assert plan.startswith(f"score_topk_f32_lds<{waves} waves"), plan


@pytest.mark.parametrize("B,I,d,k,per", [(1000, 50_000, 64, 20, 30), (3000, 20_011, 256, 20, 50),
                                         (777, 40_000, 128, 32, 10), (5000, 30_000, 192, 1, 40)])
def test_f32_split_mode(B, I, d, k, per):
    plan = ops.score_topk_plan(B, I, d, torch.float32, k)
    assert plan.startswith("score_topk_f32_lds") and "split" in plan, plan
    g = torch.Generator(device=DEV).manual_seed(B + d)
    Q = torch.randn(B, d, device=DEV, generator=g) / 8
    items = torch.randn(I, d, device=DEV, generator=g) / 8
    mask = _mask(B, I, per, g)
    idx, val = lgx.score_topk(Q, items, k, mask=mask)
    _check(Q, items, idx, val, mask, torch.arange(0, B, max(1, B // 600), device=DEV), k)


def test_f32_eight_waves_only_where_they_do_not_split():
    """d <= 128: 256-user workgroups, unless halving the user tiles alone would turn a single catalog
    sweep into a split launch -- then the 4-wave walk without splits (the Gowalla shape)."""
    gow = ops.score_topk_plan(27_522, 40_981, 64, torch.float32, 20)
    assert gow.startswith("score_topk_f32_lds<4 waves + 4 producers, 64-item tiles, 16x16x4> users[0,27522) "
                          "full-sweep") and \
        "n_splits=1" in gow and ";" not in gow, gow
    amz = ops.score_topk_plan(52_643, 91_599, 128, torch.float32, 20)
    assert amz == "score_topk_f32_lds<8 waves, 64-item tiles, 16x16x4> users[0,52643) full-sweep n_splits=1 utiles=206", amz
    assert ops.score_topk_plan(2_000, 50_000, 64, torch.float32, 20).startswith("score_topk_f32_lds<8 waves")


@pytest.mark.parametrize("d,waves", [(256, 4), (128, 8), (64, 8)])
def test_f32_full_sweep_with_split_tail_and_user_rows(d, waves):
    """256 full user tiles plus a 40-tile partial round (its own split launch), user_rows permuting a
    larger query table, masked: the 4-wave walk (d = 256, 128-user tiles) and the staggered 8-wave
    walk (d <= 128, 256-user tiles)."""
    B, I, k = 32 * waves * (256 + 40), 30_000, 20
    plan = ops.score_topk_plan(B, I, d, torch.float32, k)
    assert "full-sweep" in plan and plan.count(f"score_topk_f32_lds<{waves} waves") == 2, plan
    g = torch.Generator(device=DEV).manual_seed(3)
    Q = torch.randn(B + 500, d, device=DEV, generator=g) / 8
    items = torch.randn(I, d, device=DEV, generator=g) / 8
    rows = torch.randperm(B + 500, device=DEV, generator=g)[:B]
    mask = _mask(B, I, 50, g)
    idx, val = lgx.score_topk(Q, items, k, user_rows=rows, mask=mask)
    full = 32 * waves * 256
    sel = torch.cat([torch.randint(0, full, (600,), device=DEV, generator=g),
                     torch.randint(full, B, (600,), device=DEV, generator=g)])
    _check(Q, items, idx, val, mask, sel, k, user_rows=rows)


def test_f32_seeded_stages_equal_one_sweep_and_float64():
    """>= 262 144 items: the sweep runs in seeded stages; the lists equal (as sets) the unseeded
    one-launch min / max variant and the float64 top-k; min / max equal the float64 extremes."""
    B, I, d, k = 256 * 256, 300_000, 128, 20
    plan = ops.score_topk_plan(B, I, d, torch.float32, k)
    assert "full-sweep (seeded in stages)" in plan and plan.startswith("score_topk_f32_lds<8 waves"), plan
    g = torch.Generator(device=DEV).manual_seed(5)
    Q = torch.randn(B, d, device=DEV, generator=g) / 8
    items = torch.randn(I, d, device=DEV, generator=g) / 8
    mask = _mask(B, I, 40, g)
    idx, val = lgx.score_topk(Q, items, k, mask=mask)
    idx1, val1, mm = lgx.score_topk(Q, items, k, mask=mask, want_minmax=True)
    ka, kb = torch.sort(idx.long(), 1), torch.sort(idx1.long(), 1)
    assert torch.equal(ka.values, kb.values), "seeded lists differ from the one-launch sweep"
    assert torch.equal(val.gather(1, ka.indices), val1.gather(1, kb.indices))
    _check(Q, items, idx, val, mask, torch.randint(0, B, (1000,), device=DEV, generator=g), k)
    lo, hi = float("inf"), float("-inf")
    for u0 in range(0, B, 2048):
        S = Q[u0:u0 + 2048].double() @ items.double().T
        lo, hi = min(lo, S.min().item()), max(hi, S.max().item())
    m = mm.cpu().numpy().astype(np.float64)
    assert abs(m[0] - lo) <= 1e-5 * abs(lo) + 1e-6 and abs(m[1] - hi) <= 1e-5 * abs(hi) + 1e-6, (m, lo, hi)


def test_f32_sigmoid_and_mask_value_like_procedure_test():
    """Procedure.Test's call: sigmoid scores, positives at -(1 << 10); a user with every item but
    3 masked gets those 3 then the masked tail (mask_value, the masked items in order)."""
    B, I, d, k = 300, 5000, 64, 20
    g = torch.Generator(device=DEV).manual_seed(8)
    Q = torch.randn(B, d, device=DEV, generator=g) / 8
    items = torch.randn(I, d, device=DEV, generator=g) / 8
    lists = [sorted(set(torch.randint(0, I, (30,), generator=torch.Generator().manual_seed(u)).tolist()))
             for u in range(B)]
    lists[7] = [i for i in range(I) if i not in (5, 77, 4000)]
    mask = ops.lists_to_device_csr(lists, DEV)
    idx, val = lgx.score_topk(Q, items, k, mask=mask, mask_value=-float(1 << 10), apply_sigmoid=True)
    assert sorted(idx[7, :3].tolist()) == [5, 77, 4000]
    assert (val[7, 3:] == -1024.0).all() and idx[7, 3:].tolist() == lists[7][:k - 3]
    S = torch.sigmoid((Q.double() @ items.double().T))
    for u in (0, 1, 100, 299):
        S[u, torch.tensor(lists[u], device=DEV)] = -1.0
        want = torch.topk(S[u], k).values
        assert torch.allclose(val[u].double(), want, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("dtype,B,I,d,rows", [(torch.float32, 16384, 100_003, 64, False),
                                              (torch.float32, 333, 50_000, 256, True),
                                              (torch.float32, 1000, 20_000, 96, False),     # top-1 fall-back
                                              (torch.bfloat16, 40_000, 70_001, 128, False),
                                              (torch.bfloat16, 77, 5_000, 256, True)])
def test_score_minmax_vs_float64(dtype, B, I, d, rows):
    """lgx_score_minmax (np.max / np.min of the full dot matrix, recommend.py:163-164, :377): the
    LDS walk's min / max mode (f32 and bf16, full-sweep and split plans, padding users, a ragged
    last tile, user_rows) and the top-1 fall-back, against float64 on the device."""
    g = torch.Generator(device=DEV).manual_seed(B + d)
    n_q = B + 100 if rows else B
    Q = (torch.randn(n_q, d, device=DEV, generator=g) / 8).to(dtype)
    items = (torch.randn(I, d, device=DEV, generator=g) / 8).to(dtype)
    user_rows = torch.randperm(n_q, device=DEV, generator=g)[:B] if rows else None
    mm = ops.score_minmax(Q, items, user_rows=user_rows).cpu().numpy().astype(np.float64)
    Qs = Q[user_rows] if rows else Q
    lo, hi = float("inf"), float("-inf")
    for u0 in range(0, B, 2048):
        S = Qs[u0:u0 + 2048].double() @ items.double().T
        lo, hi = min(lo, S.min().item()), max(hi, S.max().item())
    assert abs(mm[0] - lo) <= 1e-5 * abs(lo) + 1e-6 and abs(mm[1] - hi) <= 1e-5 * abs(hi) + 1e-6, (mm, lo, hi)


@pytest.mark.parametrize("B,I,k,rows", [(30_001, 33_333, 7, True), (26_000, 20_011, 24, False),
                                        (28_123, 41_000, 1, True), (27_522, 40_981, 20, False),
                                        (40_000, 300_000, 20, True)])
def test_f32_producer_consumer_walk_equals_the_four_wave_walk(B, I, k, rows):
    """fp32 d = 64 with a 128-user tile plan (the Gowalla shape's): the producer / consumer walk
    (4 MFMA waves hand their scores through LDS to 4 top-k waves) against the 4-wave walk of the min/max
    variant on the same inputs -- lists equal as sets with their values, bit for bit.  Padding users,
    a catalog tail, user_rows, k = 1 / 7 / 20 / 24 (the largest whose lists fit beside the score
    buffers; k = 32 keeps the 4-wave walk), a 300 K-item catalog swept in seeded stages (each stage's
    lists seed the next) with a split tail range, and masks that take out each user's best items
    (exact searches and parked suspects) plus random ones."""
    d = 64
    plan = ops.score_topk_plan(B, I, d, torch.float32, k)
    assert plan.startswith("score_topk_f32_lds<4 waves + 4 producers") and "n_splits=1" in plan, plan
    assert ops.score_topk_plan(B, I, d, torch.float32, 32).startswith("score_topk_f32_lds<4 waves, ")
    g = torch.Generator(device=DEV).manual_seed(B + k)
    n_q = B + 777 if rows else B
    Q = torch.randn(n_q, d, device=DEV, generator=g) / 8
    items = torch.randn(I, d, device=DEV, generator=g) / 8
    user_rows = torch.randperm(n_q, device=DEV, generator=g)[:B] if rows else None
    Qu = Q[user_rows] if rows else Q
    best = torch.cat([torch.topk(Qu[u0:u0 + 2048] @ items.T, 40, dim=1).indices for u0 in range(0, B, 2048)])
    m = torch.cat([best[:, ::2], torch.randint(0, I, (B, 30), device=DEV, generator=g)], 1).sort(1).values
    keep = torch.ones_like(m, dtype=torch.bool)
    keep[:, 1:] = m[:, 1:] != m[:, :-1]
    indptr = torch.zeros(B + 1, dtype=torch.int64, device=DEV)
    indptr[1:] = torch.cumsum(keep.sum(1), 0)
    mask = (indptr, m[keep].to(torch.int32))
    idx, val = lgx.score_topk(Q, items, k, user_rows=user_rows, mask=mask)
    idx1, val1, _ = lgx.score_topk(Q, items, k, user_rows=user_rows, mask=mask, want_minmax=True)
    ka, kb = torch.sort(idx.long(), 1), torch.sort(idx1.long(), 1)
    assert torch.equal(ka.values, kb.values), "producer/consumer lists differ from the 4-wave walk"
    assert torch.equal(val.gather(1, ka.indices), val1.gather(1, kb.indices))
    assert (idx >= 0).all()
    users = torch.repeat_interleave(torch.arange(B, device=DEV), indptr[1:] - indptr[:-1])
    got = torch.arange(B, device=DEV)[:, None] * I + idx.long()
    assert not torch.isin(got, users * I + mask[1].long()).any(), "a masked item was returned"
