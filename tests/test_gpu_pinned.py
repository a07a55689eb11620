"""GPU: the exact kernel instantiations bench.py times, pinned against the oracle.

bench.py's numbers rest on three dispatches; each test below first asserts (through the host-only
introspection entry points lgx_spmm_kernel_name / lgx_score_topk_plan) that it runs the SAME
instantiation / launch plan as the benchmark configuration, then checks the result:

  * C4 propagation (BASELINE configs[3], bench default): spmm_segments<bf16,16,1,16> -- d=128 bf16,
    the seg_len > 128 plan -- and its fp32 twin spmm_segments<f32,32,1,8>, on a hub-heavy graph with
    seg_len 8192 forced (split rows + fix-up) against oracle.propagate; and the full-size 10M x 1M
    graph at d=128 in both dtypes through the eigenvector property.
  * C5 scoring (configs[4]): the LDS kernel in full-sweep mode plus the catalog-split tail launch,
    d=256 bf16, mask on, checked on the device against float64 scores for sampled users.
  * C1 (configs[0], Gowalla shape 29,858 x 40,981, 810,128 edges, K=3, d=64 fp32): adjacency
    bit-exact and propagation against the oracle.

Tolerances as tests/test_gpu_parity.py: fp32 |gpu - oracle| <= 1e-5 |oracle| + 1e-6 max|E0|;
bf16 storage <= 2e-2 |oracle| + 2e-2 rms(oracle); top-k: k distinct unmasked items, each within
1e-5 of the exact k-th best (reference: model.py:163-176, Procedure.py:127-135).
"""
import re

import numpy as np
import pytest
import torch

from oracle import oracle

import factors_of_serendipity_recommendation_amd as lgx
from factors_of_serendipity_recommendation_amd import ops
from factors_of_serendipity_recommendation_amd.graph import choose_seg_len
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_edges, synth_graph

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
C4 = CONFIGS["synth10m"]


def _bf16_round(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).to(torch.float32).numpy()


def _bench_spmm_kernel(dtype):
    return ops.spmm_kernel_name(C4.d, dtype, choose_seg_len(2 * C4.n_edges))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_c4_spmm_instantiation_on_hub_graph(dtype):
    """The C4 kernel (d=128, seg_len 8192) on a graph whose hub rows are split into many segments."""
    rng = np.random.default_rng(404)
    U, I, E, d = 100_000, 4_000, 1_500_000, C4.d
    u = rng.integers(0, U, E).astype(np.int32)
    i = (rng.zipf(1.3, E) % I).astype(np.int32)
    ip, ix, iv = oracle.build_norm_adj(u, i, U, I, dedup=True)
    seg = choose_seg_len(2 * C4.n_edges)
    A = lgx.from_csr_arrays(ip, ix, iv, device=DEV, n_users=U, n_items=I, seg_len=seg)
    assert A.plan.seg_len == seg == 8192
    assert int(np.diff(ip).max()) > 4 * seg and len(A.plan.split_row) > 0  # hub rows take the fix-up
    assert ops.spmm_kernel_name(d, dtype, A.plan.seg_len) == _bench_spmm_kernel(dtype)
    E0 = (rng.standard_normal((U + I, d)) * 0.1).astype(np.float32)
    if dtype == torch.bfloat16:
        E0 = _bf16_round(E0)
    out = lgx.propagate(A, torch.from_numpy(E0).to(DEV).to(dtype), C4.K).cpu().numpy()
    ref = oracle.propagate(ip, ix, iv, E0, C4.K)
    err = np.abs(out - ref)
    if dtype == torch.bfloat16:
        tol = 2e-2 * np.abs(ref) + 2e-2 * np.sqrt(np.mean(ref ** 2))
    else:
        tol = 1e-5 * np.abs(ref) + 1e-6 * np.abs(E0).max()
    assert (err <= tol).all(), f"max err {err.max():.3e}"


@pytest.mark.slow
def test_c4_full_size_d128_both_dtypes():
    """BASELINE configs[3] at full size (10M x 1M, 1e9 nonzeros) and the bench's d=128, in the bench's
    bf16 storage and in fp32: v = sqrt(deg) is a fixed point of A^ (A^ v = v), so every layer and the
    layer mean reproduce v column-scaled; rows of degree 0 give 0."""
    A = synth_graph(C4, 2020, DEV)
    assert A.nnz == 2 * C4.n_edges
    deg = torch.diff(A.indptr).double()
    v = deg.sqrt()
    col = torch.arange(1, C4.d + 1, device=DEV, dtype=torch.float64) / C4.d
    for dtype, rel in ((torch.bfloat16, 2e-2), (torch.float32, 1e-4)):
        assert ops.spmm_kernel_name(C4.d, dtype, A.plan.seg_len) == _bench_spmm_kernel(dtype)
        E0 = (v[:, None] * col[None, :]).to(dtype)
        out = lgx.propagate(A, E0, C4.K)
        ref = E0.float()
        bad = ((out - ref).abs() > rel * ref.abs() + rel * 1e-3).sum().item()
        assert bad == 0, f"{dtype}: {bad} entries off the fixed point"
        del E0, out, ref
        torch.cuda.empty_cache()


def test_c5_scoring_full_sweep_plan_d256():
    """The C5 launch plan (full-sweep LDS kernel over whole rounds of 256 user tiles, then a
    catalog-split launch for the 67-tile remainder) at d=256 bf16 with the train mask."""
    B, I, d, k = 256 * (256 + 67), 100_000, 256, 20
    plan = ops.score_topk_plan(B, I, d, torch.bfloat16, k)
    # the bench's 1M-item catalog seeds its full sweep (test_seeded_full_sweep_equals_one_sweep)
    # the bench's 1M-item catalog is pinned at full size by test_c5_full_catalog_1m_items_bench_plan
    bench = ops.score_topk_plan(1_000_000, 1_000_000, d, torch.bfloat16, k).replace(" (seeded in stages)", "")
    # score floors need splits of >= 65 536 items: the 1M catalog's tail splits take them, 100 K's do not
    plan, bench = plan.replace(" (score floors)", ""), bench.replace(" (score floors)", "")
    kinds = [p.split(" users")[0] + " " + p.split(") ")[1].split(" n_splits")[0] for p in plan.split("; ")]
    bkinds = [p.split(" users")[0] + " " + p.split(") ")[1].split(" n_splits")[0] for p in bench.split("; ")]
    assert kinds == bkinds and "full-sweep" in plan and len(kinds) == 2, (plan, bench)
    g = torch.Generator(device=DEV).manual_seed(11)
    Q = (torch.randn(B, d, device=DEV, generator=g) / 16).bfloat16()
    items = (torch.randn(I, d, device=DEV, generator=g) / 16).bfloat16()
    per = 50
    m = torch.randint(0, I, (B, per), device=DEV, generator=g).sort(1).values
    keep = torch.ones_like(m, dtype=torch.bool)
    keep[:, 1:] = m[:, 1:] != m[:, :-1]
    lens = keep.sum(1)
    indptr = torch.zeros(B + 1, dtype=torch.int64, device=DEV)
    indptr[1:] = torch.cumsum(lens, 0)
    mask = (indptr, m[keep].to(torch.int32))
    idx, val = lgx.score_topk(Q, items, k, mask=mask)
    # users from both launches (full-sweep range and the split tail), checked in float64
    sel = torch.cat([torch.randint(0, 65536, (1500,), device=DEV, generator=g),
                     torch.randint(65536, B, (1500,), device=DEV, generator=g)])
    S = Q[sel].double() @ items.double().T
    for j, u in enumerate(sel.tolist()):
        S[j, mask[1][indptr[u]:indptr[u + 1]].long()] = float("-inf")
    kth = torch.topk(S, k, dim=1).values[:, -1:]
    got_idx = idx[sel].long()
    assert (got_idx >= 0).all()
    got = S.gather(1, got_idx)
    assert torch.isfinite(got).all()
    assert (got >= kth - 1e-5 * kth.abs().clamp(min=1.0)).all()
    srt = got_idx.sort(1).values
    assert (srt[:, 1:] != srt[:, :-1]).all()
    assert torch.allclose(val[sel].double(), got, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n_top,n_rand", [(10, 40), (40, 200)])
def test_full_sweep_masks_on_the_top_items(n_top, n_rand):
    """Full-sweep LDS kernel with every user's mask holding its own n_top best items plus n_rand
    random ones: the masked items are exactly the candidates the sweep meets first-hand, and at
    240 masked items the 256-bit Bloom filter passes nearly every survivor, so the parked-key slots
    overflow into the immediate exact search.  Result: the exact top-k of the unmasked items."""
    B, I, d, k = 256 * 256, 20_000, 256, 20
    assert "full-sweep" in ops.score_topk_plan(B, I, d, torch.bfloat16, k)
    g = torch.Generator(device=DEV).manual_seed(23)
    Q = (torch.randn(B, d, device=DEV, generator=g) / 16).bfloat16()
    items = (torch.randn(I, d, device=DEV, generator=g) / 16).bfloat16()
    tops = []
    for u0 in range(0, B, 8192):
        s = Q[u0:u0 + 8192].float() @ items.float().T
        tops.append(torch.topk(s, n_top, dim=1).indices)
    top = torch.cat(tops)
    m = torch.cat([top, torch.randint(0, I, (B, n_rand), device=DEV, generator=g)], 1).sort(1).values
    keep = torch.ones_like(m, dtype=torch.bool)
    keep[:, 1:] = m[:, 1:] != m[:, :-1]
    indptr = torch.zeros(B + 1, dtype=torch.int64, device=DEV)
    indptr[1:] = torch.cumsum(keep.sum(1), 0)
    mask = (indptr, m[keep].to(torch.int32))
    idx, val = lgx.score_topk(Q, items, k, mask=mask)
    sel = torch.randint(0, B, (2000,), device=DEV, generator=g)
    S = Q[sel].double() @ items.double().T
    for j, u in enumerate(sel.tolist()):
        S[j, mask[1][indptr[u]:indptr[u + 1]].long()] = float("-inf")
    kth = torch.topk(S, k, dim=1).values[:, -1:]
    got_idx = idx[sel].long()
    assert (got_idx >= 0).all()
    got = S.gather(1, got_idx)
    assert torch.isfinite(got).all(), "a masked item was returned"
    assert (got >= kth - 1e-5 * kth.abs().clamp(min=1.0)).all()
    srt = got_idx.sort(1).values
    assert (srt[:, 1:] != srt[:, :-1]).all()
    assert torch.allclose(val[sel].double(), got, rtol=1e-5, atol=1e-5)


def test_seeded_full_sweep_equals_one_sweep():
    """Catalogs of >= 262 144 items run the full sweep in stages ([0, 16384), [16384, 32768), ...
    doubling, then the rest), each seeding the next.  Masks put every user's own best first-stage items (and random
    ones everywhere) out of play.  The lists must equal, as sets, the one-launch sweep
    (the min/max variant never seeds) and the float64 top-k of the unmasked items."""
    B, I, d, k = 256 * 256, 300_000, 256, 20
    plan = ops.score_topk_plan(B, I, d, torch.bfloat16, k)
    assert "full-sweep (seeded in stages)" in plan, plan
    g = torch.Generator(device=DEV).manual_seed(29)
    Q = (torch.randn(B, d, device=DEV, generator=g) / 16).bfloat16()
    items = (torch.randn(I, d, device=DEV, generator=g) / 16).bfloat16()
    tops = []
    for u0 in range(0, B, 8192):
        s = Q[u0:u0 + 8192].float() @ items[:16384].float().T
        tops.append(torch.topk(s, 8, dim=1).indices)
    m = torch.cat([torch.cat(tops), torch.randint(0, I, (B, 40), device=DEV, generator=g)], 1).sort(1).values
    keep = torch.ones_like(m, dtype=torch.bool)
    keep[:, 1:] = m[:, 1:] != m[:, :-1]
    indptr = torch.zeros(B + 1, dtype=torch.int64, device=DEV)
    indptr[1:] = torch.cumsum(keep.sum(1), 0)
    mask = (indptr, m[keep].to(torch.int32))
    idx, val = lgx.score_topk(Q, items, k, mask=mask)
    idx1, val1, _ = lgx.score_topk(Q, items, k, mask=mask, want_minmax=True)
    ka = torch.sort(idx.long(), 1)
    kb = torch.sort(idx1.long(), 1)
    assert torch.equal(ka.values, kb.values), "seeded lists differ from the one-launch sweep"
    assert torch.equal(val.gather(1, ka.indices), val1.gather(1, kb.indices))
    sel = torch.randint(0, B, (1500,), device=DEV, generator=g)
    S = Q[sel].double() @ items.double().T
    for j, u in enumerate(sel.tolist()):
        S[j, mask[1][indptr[u]:indptr[u + 1]].long()] = float("-inf")
    kth = torch.topk(S, k, dim=1).values[:, -1:]
    got = S.gather(1, idx[sel].long())
    assert torch.isfinite(got).all(), "a masked item was returned"
    assert (got >= kth - 1e-5 * kth.abs().clamp(min=1.0)).all()


@pytest.mark.parametrize("mode,dtype", [("full-sweep", torch.bfloat16), ("split", torch.bfloat16),
                                        ("full-sweep", torch.float32), ("split", torch.float32)])
def test_score_floors_with_ties_and_masked_group_maxima(mode, dtype):
    """Score floors (kFloorOnly, bf16; the fp32 cases pin the unfloored walk on the same data): every
    unseeded bf16 LDS sweep -- the first seeded stage, or each split
    of a split launch -- starts its lists at the k-th largest of 64 group maxima over its first
    16384 items, groups holding a masked item dropped.  The catalog repeats 4096 distinct rows at
    random positions, so a user's best scores come in exact ties spread over many groups; the mask
    takes out every copy of the user's best row inside each floor window (so the floor must drop
    those groups) plus random items.  Lists equal, as sets with their values, the unfloored
    one-launch sweep (the min/max variant runs without floors and seeds)."""
    d, k = 64, 20
    if mode == "full-sweep":
        B, I, wins = 256 * 256, 300_000, [(0, 16384)]
    else:
        B, I = 18 * 256, 1_000_000
    plan = ops.score_topk_plan(B, I, d, dtype, k)
    if mode == "full-sweep":
        assert "full-sweep (seeded in stages)" in plan, plan
    else:
        ns = int(re.search(r"n_splits=(\d+)", plan).group(1))
        assert "full-sweep" not in plan and "split" in plan and ns > 1, plan
        per = -(-(-(-I // 64)) // ns) * 64  # the plan's split_items: whole 64-item tiles per split
        assert per >= 4 * 16384  # long enough to take floors
        wins = [(s * per, min(I, s * per + 16384)) for s in range(ns)]
    g = torch.Generator(device=DEV).manual_seed(61)
    Q = (torch.randn(B, d, device=DEV, generator=g) / 8).to(dtype)
    base = (torch.randn(4096, d, device=DEV, generator=g) / 8).to(dtype)
    rowid = torch.randint(0, 4096, (I,), device=DEV, generator=g)
    items = base[rowid].contiguous()
    best = torch.cat([(Q[u0:u0 + 8192].float() @ base.float().T).argmax(1) for u0 in range(0, B, 8192)])
    parts = [torch.randint(0, I, (B, 30), device=DEV, generator=g)]
    for lo, hi in wins:  # every copy of the user's best row inside the window
        order = torch.argsort(rowid[lo:hi])
        srt = rowid[lo:hi][order]
        s0 = torch.searchsorted(srt, best)
        s1 = torch.searchsorted(srt, best, right=True)
        j = s0[:, None] + torch.arange(int((s1 - s0).max()), device=DEV)[None, :]
        parts.append(torch.where(j < s1[:, None], lo + order[j.clamp(max=hi - lo - 1)], -1))
    m = torch.cat(parts, 1).sort(1).values
    keep = m >= 0
    keep[:, 1:] &= m[:, 1:] != m[:, :-1]
    indptr = torch.zeros(B + 1, dtype=torch.int64, device=DEV)
    indptr[1:] = torch.cumsum(keep.sum(1), 0)
    mask = (indptr, m[keep].to(torch.int32))
    idx, val = lgx.score_topk(Q, items, k, mask=mask)
    idx1, val1, _ = lgx.score_topk(Q, items, k, mask=mask, want_minmax=True)
    ka, kb = torch.sort(idx.long(), 1), torch.sort(idx1.long(), 1)
    assert torch.equal(ka.values, kb.values), "floored lists differ from the unfloored sweep"
    assert torch.equal(val.gather(1, ka.indices), val1.gather(1, kb.indices))
    assert (idx >= 0).all()
    # no masked item comes back (keys u * I + item)
    users = torch.repeat_interleave(torch.arange(B, device=DEV), indptr[1:] - indptr[:-1])
    got = torch.arange(B, device=DEV)[:, None] * I + idx.long()
    assert not torch.isin(got, users * I + mask[1].long()).any(), "a masked item was returned"


@pytest.mark.parametrize("B,I,d", [(27_522, 40_981, 64), (3_000, 100_000, 256), (2_000, 100_000, 192)])
def test_f32_score_floors_at_evaluation_shapes(B, I, d):
    """fp32 score floors (the 4-wave walk, catalogs under 262 144 items: the evaluation shapes of
    Procedure.Test / batch_test): every split takes its floor over its first eighth.  The catalog repeats
    2048 distinct rows, so a user's best scores come in exact ties spread over many floor groups, and the
    mask takes out every copy of the user's best row plus random items.  Lists equal, as sets with their
    values, the unfloored sweep of the min/max variant; no masked item comes back."""
    k = 20
    plan = ops.score_topk_plan(B, I, d, torch.float32, k)
    assert plan.startswith("score_topk_f32_lds<4 waves") and "(score floors)" in plan, plan
    g = torch.Generator(device=DEV).manual_seed(B + d)
    Q = torch.randn(B, d, device=DEV, generator=g) / 8
    base = torch.randn(2048, d, device=DEV, generator=g) / 8
    rowid = torch.randint(0, 2048, (I,), device=DEV, generator=g)
    items = base[rowid].contiguous()
    best = torch.cat([(Q[u0:u0 + 4096] @ base.T).argmax(1) for u0 in range(0, B, 4096)])
    order = torch.argsort(rowid)
    srt = rowid[order]
    s0, s1 = torch.searchsorted(srt, best), torch.searchsorted(srt, best, right=True)
    j = s0[:, None] + torch.arange(int((s1 - s0).max()), device=DEV)[None, :]
    copies = torch.where(j < s1[:, None], order[j.clamp(max=I - 1)], -1)
    m = torch.cat([copies, torch.randint(0, I, (B, 25), device=DEV, generator=g)], 1).sort(1).values
    keep = m >= 0
    keep[:, 1:] &= m[:, 1:] != m[:, :-1]
    indptr = torch.zeros(B + 1, dtype=torch.int64, device=DEV)
    indptr[1:] = torch.cumsum(keep.sum(1), 0)
    mask = (indptr, m[keep].to(torch.int32))
    idx, val = lgx.score_topk(Q, items, k, mask=mask)
    idx1, val1, _ = lgx.score_topk(Q, items, k, mask=mask, want_minmax=True)
    ka, kb = torch.sort(idx.long(), 1), torch.sort(idx1.long(), 1)
    assert torch.equal(ka.values, kb.values), "floored lists differ from the unfloored sweep"
    assert torch.equal(val.gather(1, ka.indices), val1.gather(1, kb.indices))
    users = torch.repeat_interleave(torch.arange(B, device=DEV), indptr[1:] - indptr[:-1])
    got = torch.arange(B, device=DEV)[:, None] * I + idx.long()
    assert not torch.isin(got, users * I + mask[1].long()).any(), "a masked item was returned"


@pytest.mark.parametrize("d,k,rows", [(64, 1, False), (128, 7, True), (128, 32, False), (256, 20, True),
                                      (96, 20, True)])
def test_seeded_sweep_shapes(d, k, rows):
    """The seeded stages across the LDS kernel's shapes (d, k) and with user_rows: lists equal, as
    sets, the one-launch sweep of the unseeded min/max variant."""
    B, I = 256 * 256, 270_000
    assert "seeded in stages" in ops.score_topk_plan(B, I, d, torch.bfloat16, k)
    g = torch.Generator(device=DEV).manual_seed(31 + d + k)
    n_q = B + 1000 if rows else B
    Q = (torch.randn(n_q, d, device=DEV, generator=g) / 16).bfloat16()
    items = (torch.randn(I, d, device=DEV, generator=g) / 16).bfloat16()
    user_rows = torch.randperm(n_q, device=DEV, generator=g)[:B] if rows else None
    m = torch.randint(0, I, (B, 30), device=DEV, generator=g).sort(1).values
    keep = torch.ones_like(m, dtype=torch.bool)
    keep[:, 1:] = m[:, 1:] != m[:, :-1]
    indptr = torch.zeros(B + 1, dtype=torch.int64, device=DEV)
    indptr[1:] = torch.cumsum(keep.sum(1), 0)
    mask = (indptr, m[keep].to(torch.int32))
    idx, val = lgx.score_topk(Q, items, k, user_rows=user_rows, mask=mask)
    idx1, val1, _ = lgx.score_topk(Q, items, k, user_rows=user_rows, mask=mask, want_minmax=True)
    ka, kb = torch.sort(idx.long(), 1), torch.sort(idx1.long(), 1)
    assert torch.equal(ka.values, kb.values), "seeded lists differ from the one-launch sweep"
    assert torch.equal(val.gather(1, ka.indices), val1.gather(1, kb.indices))
    assert (idx >= 0).all()


def test_c1_gowalla_shape_vs_oracle():
    cfg = CONFIGS["gowalla"]
    u, i = synth_edges(cfg, 2020, DEV)
    assert u.numel() == cfg.n_edges
    A = lgx.build_norm_adj(u, i, cfg.n_users, cfg.n_items, dedup=True, device=DEV)
    ip, ix, iv = oracle.build_norm_adj(u.cpu().numpy(), i.cpu().numpy(), cfg.n_users, cfg.n_items, dedup=True)
    assert np.array_equal(A.indptr.cpu().numpy(), ip) and np.array_equal(A.indices.cpu().numpy(), ix)
    assert np.array_equal(A.vals.cpu().numpy(), iv)
    E0 = lgx.fill_normal((cfg.n_users + cfg.n_items, cfg.d), 0.1, 2020, device=DEV)
    out = lgx.propagate(A, E0, cfg.K).cpu().numpy()
    ref = oracle.propagate(ip, ix, iv, E0.cpu().numpy(), cfg.K)
    err = np.abs(out - ref)
    assert (err <= 1e-5 * np.abs(ref) + 1e-6 * float(E0.abs().max())).all(), f"max err {err.max():.3e}"


def test_c3_amazon_full_size_d128_vs_oracle():
    """C3 (configs[2]: 52,643 x 91,599, 2,984,108 edges, K=4, d=128) at full size against the f64
    oracle: fp32 storage at the north-star tolerance and bf16 storage (the config's dtype) at the
    bf16 tolerance, from the same bf16-representable E0."""
    cfg = CONFIGS["amazon"]
    u, i = synth_edges(cfg, 2020, DEV)
    A = lgx.build_norm_adj(u, i, cfg.n_users, cfg.n_items, dedup=True, device=DEV)
    ip, ix, iv = A.indptr.cpu().numpy(), A.indices.cpu().numpy(), A.vals.cpu().numpy()
    E0 = lgx.fill_normal((cfg.n_users + cfg.n_items, cfg.d), 0.1, 2020, device=DEV).to(torch.bfloat16)
    ref = oracle.propagate(ip, ix, iv, E0.float().cpu().numpy(), cfg.K)
    out32 = lgx.propagate(A, E0.float(), cfg.K).cpu().numpy()
    err = np.abs(out32 - ref)
    assert (err <= 1e-5 * np.abs(ref) + 1e-6 * float(E0.float().abs().max())).all(), f"fp32 max err {err.max():.3e}"
    out16 = lgx.propagate(A, E0, cfg.K).cpu().numpy()
    assert (np.abs(out16 - ref) <= 2e-2 * np.abs(ref) + 2e-2 * np.sqrt(np.mean(ref ** 2))).all()


def _plan_kinds(plan):
    """Per launch of a plan string: kernel, mode (seeding included) and n_splits; user ranges and
    tile counts (which scale with the batch) dropped."""
    out = []
    for p in plan.split("; "):
        kernel = p.split(" users")[0]
        mode = p.split(") ", 1)[1].split(" utiles")[0]
        out.append(kernel + " " + mode)
    return out


def _masked_topk_check(Q, items, idx, val, mask, sel, k, chunk=250):
    """sel users against float64 scores on the device, in chunks: k distinct unmasked items, each
    within 1e-5 of the exact k-th best, values equal to the float64 scores to 1e-5."""
    indptr, mi = mask
    items64 = items.double()
    for c0 in range(0, sel.numel(), chunk):
        s = sel[c0:c0 + chunk]
        S = Q[s].double() @ items64.T
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
        del S


def test_c5_full_catalog_1m_items_bench_plan():
    """BASELINE configs[4] at its own catalog: 82,688 users x 1,000,000 items, d=256 bf16, top-20,
    50 masked items per user.  The launch plan is the bench's (1 M users) launch for launch: the
    full sweep seeded in stages (7 launches over [0,16384), ..., [524288, 1M)) and the catalog-split
    tail with 3 splits -- "seeded" included in the comparison.  1,500 users of each launch are
    checked against float64 scores on the device."""
    B, I, d, k = 256 * (256 + 67), 1_000_000, 256, 20
    plan = ops.score_topk_plan(B, I, d, torch.bfloat16, k)
    bench = ops.score_topk_plan(1_000_000, I, d, torch.bfloat16, k)
    assert _plan_kinds(plan) == _plan_kinds(bench), (plan, bench)
    assert "full-sweep (seeded in stages)" in plan and len(_plan_kinds(plan)) == 2
    g = torch.Generator(device=DEV).manual_seed(55)
    Q = (torch.randn(B, d, device=DEV, generator=g) / 16).bfloat16()
    items = (torch.randn(I, d, device=DEV, generator=g) / 16).bfloat16()
    m = torch.randint(0, I, (B, 50), device=DEV, generator=g).sort(1).values
    keep = torch.ones_like(m, dtype=torch.bool)
    keep[:, 1:] = m[:, 1:] != m[:, :-1]
    indptr = torch.zeros(B + 1, dtype=torch.int64, device=DEV)
    indptr[1:] = torch.cumsum(keep.sum(1), 0)
    mask = (indptr, m[keep].to(torch.int32))
    idx, val = lgx.score_topk(Q, items, k, mask=mask)
    sel = torch.cat([torch.randint(0, 65536, (1500,), device=DEV, generator=g),
                     torch.randint(65536, B, (1500,), device=DEV, generator=g)])
    _masked_topk_check(Q, items, idx, val, mask, sel, k)


def test_c5_fp32_scoring_leg_plan_and_values():
    """The fp32 scoring leg of the bench (the reference's precision, model.py:183, Procedure.py:127-135)
    on the bench's own launch plan: f32 query and item tables through score_topk_f32_lds (16x16x4 f32
    MFMA, 4 waves x 32 users per workgroup at d=256), x 1,000,000 items, d=256, top-20, 50 masked
    items per user.  The bench scores SURVEY C5's 1,000,000 users: 7,813 user tiles = 30 full rounds of
    the 256 resident workgroups (one full sweep seeded in stages: 7 launches over [0,16384), ...,
    [524288, 1M)) plus a 133-tile partial round, launched catalog-split.  Here 256 + 133 tiles
    (49,792 users) give the same plan launch for launch ("seeded" and n_splits included), and 1,500
    users spread over every workgroup of both launches are checked against float64 scores."""
    B, I, d, k = 128 * (256 + 133), 1_000_000, 256, 20
    plan = ops.score_topk_plan(B, I, d, torch.float32, k)
    bench = ops.score_topk_plan(1_000_000, I, d, torch.float32, k)
    assert _plan_kinds(plan) == _plan_kinds(bench), (plan, bench)
    assert len(_plan_kinds(plan)) == 2 and plan.startswith("score_topk_f32_lds<4 waves"), plan
    assert "full-sweep (seeded in stages)" in plan and "split" in plan.split("; ")[1], plan
    g = torch.Generator(device=DEV).manual_seed(57)
    Q = torch.randn(B, d, device=DEV, generator=g) / 16
    items = torch.randn(I, d, device=DEV, generator=g) / 16
    m = torch.randint(0, I, (B, 50), device=DEV, generator=g).sort(1).values
    keep = torch.ones_like(m, dtype=torch.bool)
    keep[:, 1:] = m[:, 1:] != m[:, :-1]
    indptr = torch.zeros(B + 1, dtype=torch.int64, device=DEV)
    indptr[1:] = torch.cumsum(keep.sum(1), 0)
    mask = (indptr, m[keep].to(torch.int32))
    idx, val = lgx.score_topk(Q, items, k, mask=mask)
    # every 128-user workgroup, and every wave lane position, is sampled
    nt = B // 128
    sel = torch.cat([torch.arange(0, B, 128, device=DEV) + torch.randint(0, 128, (nt,), device=DEV, generator=g),
                     torch.randint(0, B, (1500 - nt,), device=DEV, generator=g)])
    assert sel.numel() == 1500
    _masked_topk_check(Q, items, idx, val, mask, sel, k)
