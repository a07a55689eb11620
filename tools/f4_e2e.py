"""End-to-end f4 (stratified_candidates, recommend.py:314-356 shape): the call returning the lazy
CandidateLists (per-batch async copies into one pinned array) against a synchronous per-batch loop
that builds Python lists, 16384 users x 1 M items, d=64 f32, 1000 candidates per user, 4096-user
batches; train items as Python lists and as a device CSR."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from factors_of_serendipity_recommendation_amd import ops, recommend

U, I, d, B = 16384, 1_000_000, 64, 4096
g = torch.Generator(device="cuda").manual_seed(0)
Eu = torch.randn(U, d, device="cuda", generator=g) * 0.3
Ei = torch.randn(I, d, device="cuda", generator=g) * 0.3
rng = np.random.default_rng(0)
train = [np.sort(rng.choice(I, 40, replace=False)).tolist() for _ in range(U)]
targets = [1000] * U


def sync_loop():
    min16, inter16 = recommend.stratification_bounds(Eu, Ei, 10, 0.1)
    mp, mi = ops.lists_to_device_csr(train, "cuda", sort=True)
    out = []
    from factors_of_serendipity_recommendation_amd import _lib
    L = _lib.lib()
    tgt = torch.as_tensor(np.asarray(targets, dtype=np.int32), device="cuda")
    for b0 in range(0, U, B):
        b1 = min(U, b0 + B)
        lab, hist = recommend.strat_labels(Eu[b0:b1], Ei, mp[b0:], mi, min16, inter16, 10, None)
        o = torch.empty((b1 - b0, 1000), dtype=torch.int32, device="cuda")
        c = torch.empty(b1 - b0, dtype=torch.int32, device="cuda")
        _lib.check(L.lgx_strat_select(lab.data_ptr(), b1 - b0, I, hist.data_ptr(), 11, tgt[b0:b1].data_ptr(),
                                      (0 * 0x9E3779B97F4A7C15 + b0) % 2 ** 64, o.data_ptr(), 1000, c.data_ptr(),
                                      ops._stream_ptr(torch.device("cuda"))), "select")
        oc, cc = o.cpu().numpy(), c.cpu().numpy()
        out.extend(oc[j, :cc[j]].tolist() for j in range(b1 - b0))
    return out


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(reps):
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        best.append(time.perf_counter() - t)
    return r, float(np.median(best)) * 1e3


a, ms_sync = timed(sync_loop)
b, ms_pipe = timed(lambda: recommend.stratified_candidates(Eu, Ei, train, targets, seed=0, batch=B))
assert b == a, "pipelined lists differ from the synchronous loop"
csr = ops.lists_to_device_csr(train, "cuda", sort=True)
c, ms_csr = timed(lambda: recommend.stratified_candidates(Eu, Ei, csr, targets, seed=0, batch=B))
assert c == a
t = time.perf_counter()
rows = [c[u] for u in range(U)]
ms_rows = (time.perf_counter() - t) * 1e3
print(f"f4 end-to-end, {U} users x {I} items: synchronous per-batch lists {ms_sync:.1f} ms; "
      f"stratified_candidates (lazy CandidateLists) {ms_pipe:.1f} ms from Python train lists, {ms_csr:.1f} ms "
      f"from a device CSR ({U / ms_csr * 1e3:.0f} users/s); materialising every row as a list afterwards "
      f"{ms_rows:.1f} ms; lists identical", flush=True)

# component times (HIP events on the current stream): bounds pass, fused labels + counts, select
from factors_of_serendipity_recommendation_amd import _lib  # noqa: E402


def ev_time(fn, reps=3):
    fn()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    return float(np.median(out))


min16, inter16 = recommend.stratification_bounds(Eu, Ei, 10, 0.1)
mp, mi = csr
t_b = ev_time(lambda: recommend.stratification_bounds(Eu, Ei, 10, 0.1))
t_l = ev_time(lambda: recommend.strat_labels(Eu[:B], Ei, mp, mi, min16, inter16, 10, None))
lab, hist = recommend.strat_labels(Eu[:B], Ei, mp, mi, min16, inter16, 10, None)
o = torch.empty((B, 1000), dtype=torch.int32, device="cuda")
cn = torch.empty(B, dtype=torch.int32, device="cuda")
tg = torch.full((B,), 1000, dtype=torch.int32, device="cuda")
L = _lib.lib()
t_s = ev_time(lambda: _lib.check(L.lgx_strat_select(lab.data_ptr(), B, I, hist.data_ptr(), 11, tg.data_ptr(), 7,
                                                    o.data_ptr(), 1000, cn.data_ptr(),
                                                    ops._stream_ptr(torch.device("cuda"))), "select"))
print(f"f4 components per {B}-user batch: bounds pass (all {U} users) {t_b:.2f} ms, fused labels + counts "
      f"{t_l:.2f} ms, select {t_s:.2f} ms", flush=True)
