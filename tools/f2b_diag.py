"""Development: where the Gowalla-shape BPR epoch spends its time (Loader graph vs synth graph
propagation, epoch wall, epoch with host syncs per minibatch)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import ops, train  # noqa: E402
from factors_of_serendipity_recommendation_amd.dataloader import Loader  # noqa: E402
from factors_of_serendipity_recommendation_amd.model import LightGCN  # noqa: E402
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_edges, synth_graph  # noqa: E402


def ev_ms(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


cfg = CONFIGS["gowalla"]
u, i = synth_edges(cfg, 2020, "cuda")
u, i = u.cpu().numpy(), i.cpu().numpy()
path = "/tmp/f2b_diag"
os.makedirs(path, exist_ok=True)
order = np.argsort(u, kind="stable")
u, i = u[order], i[order]
bounds = np.searchsorted(u, np.arange(cfg.n_users + 1))
with open(os.path.join(path, "train.txt"), "w") as f:
    for x in range(cfg.n_users):
        if bounds[x + 1] > bounds[x]:
            f.write(str(x) + " " + " ".join(map(str, i[bounds[x]:bounds[x + 1]])) + "\n")
with open(os.path.join(path, "test.txt"), "w") as f:
    f.write(f"0 {int(i[0])}\n")
ds = Loader(path=path, device="cuda", cache_adj=False)
conf = {"latent_dim_rec": cfg.d, "lightGCN_n_layers": cfg.K, "keep_prob": 0.6, "A_split": False,
        "pretrain": 0, "dropout": 0, "decay": 1e-4, "lr": 0.001}
torch.manual_seed(0)
model = LightGCN(conf, ds).to("cuda")
A = model._csr
A.ensure_plan()
S = synth_graph(cfg, seed=2020, device="cuda")
S.ensure_plan()
for name, G in (("loader", A), ("synth", S)):
    print(f"{name}: rows {G.n_rows} nnz {G.nnz} U {G.n_users} I {G.n_items} phases {G.phases()} seg_len "
          f"{G.plan.seg_len} n_segs {len(G.plan.seg_row)} split {len(G.plan.split_row)}", flush=True)
    E0 = lgx.fill_normal((G.n_rows, cfg.d), 0.1, 7)
    print(f"  propagate K=3: {ev_ms(lambda: ops.propagate(G, E0, 3)) * 1e3:.1f} us", flush=True)
bpr = train.BPRLoss(model, conf)
for graph in (False, True, False, True):
    train.BPR_train_original(ds, model, bpr, 0, batch_size=2048, graph=graph)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    train.BPR_train_original(ds, model, bpr, 1, batch_size=2048, graph=graph)
    e1.record()
    torch.cuda.synchronize()
    print(f"epoch graph={graph}: events {e0.elapsed_time(e1):.1f} ms, host wall {(time.perf_counter() - t0) * 1e3:.1f} ms",
          flush=True)
# one minibatch, host issue time vs GPU time
us, ps, ns = [torch.randint(0, n, (2048,), device="cuda") for n in (cfg.n_users, cfg.n_items, cfg.n_items)]
model._lgx_trusted_indices = True
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    bpr.stageOne(us, ps, ns)
t_issue = (time.perf_counter() - t0) / 50
torch.cuda.synchronize()
t_all = (time.perf_counter() - t0) / 50
print(f"minibatch: host issue {t_issue * 1e3:.3f} ms, with drain {t_all * 1e3:.3f} ms", flush=True)
