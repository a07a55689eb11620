"""Seeded synthetic bipartite graphs with the shapes named in BASELINE.json (no datasets travel to
the GPU box, and Gowalla/Amazon-book train.txt are not shipped by the reference -- see
.MISSING_LARGE_BLOBS).  User degrees follow a truncated Zipf law (min 1), item popularity a Zipf
law over a random permutation of item ids; edges are de-duplicated and trimmed to exactly E.
Everything heavy runs on the GPU (lgx_synth_edges + the CSR builder); outputs are identical on
every device and rank for a given seed.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .graph import CSRGraph, _stream_ptr, build_norm_adj


@dataclass(frozen=True)
class GraphConfig:
    name: str
    n_users: int
    n_items: int
    n_edges: int
    K: int
    d: int
    dtype: str  # "f32" | "bf16"
    alpha_user: float = 1.0
    alpha_item: float = 0.9


CONFIGS = {
    # BASELINE.json configs[0]: Gowalla stats (LightGCN-tf/README.md:37-39)
    "gowalla": GraphConfig("gowalla", 29_858, 40_981, 810_128, 3, 64, "f32"),
    # configs[1]: MovieLens-1M bipartite graph, K=3 d=64 fp32
    "ml1m": GraphConfig("ml1m", 6_040, 3_706, 1_000_209, 3, 64, "f32", 0.8, 0.8),
    # configs[2]: Amazon-Book scale (README.md:77-79), K=4 d=128 bf16
    "amazon": GraphConfig("amazon", 52_643, 91_599, 2_984_108, 4, 128, "bf16"),
    # configs[3]: 10M users x 1M items, 500M edges, K=3 d=128 (bf16 perf / fp32 parity)
    "synth10m": GraphConfig("synth10m", 10_000_000, 1_000_000, 500_000_000, 3, 128, "bf16"),
}


def user_degrees(n_users: int, n_items: int, n_edges: int, alpha: float, seed: int) -> np.ndarray:
    """Truncated Zipf degrees (min 1, max n_items/2) summing to ~n_edges, shuffled over user ids."""
    rng = np.random.default_rng(seed)
    w = (np.arange(1, n_users + 1, dtype=np.float64)) ** (-alpha)
    rng.shuffle(w)
    cap = max(1, n_items // 2)
    w = w / w.sum()

    def degs(c):
        return np.minimum(cap, np.maximum(1, np.round(w * c)))

    lo, hi = 0.0, float(n_edges)
    while degs(hi).sum() < n_edges and hi < 1e15:  # the cap clips the head: scale the tail up
        hi *= 2
    for _ in range(60):  # bisection on the scale so that the clipped law sums to ~n_edges
        mid = 0.5 * (lo + hi)
        if degs(mid).sum() < n_edges:
            lo = mid
        else:
            hi = mid
    return degs(hi).astype(np.int64)


def synth_edges(cfg: GraphConfig, seed: int = 2020, device="cuda", oversample: float = 1.15):
    """(users int32 [E], items int32 [E]) on the device, exactly cfg.n_edges unique pairs."""
    device = torch.device(device)
    L = _lib.lib()
    rng = np.random.default_rng(seed + 1)
    pop = (np.arange(1, cfg.n_items + 1, dtype=np.float64)) ** (-cfg.alpha_item)
    cdf = np.cumsum(pop)
    cdf = (cdf / cdf[-1]).astype(np.float32)
    cdf[-1] = 1.0
    perm = rng.permutation(cfg.n_items).astype(np.int32)
    cdf_t = torch.from_numpy(cdf).to(device)
    perm_t = torch.from_numpy(perm).to(device)
    want = cfg.n_edges
    keys = torch.empty(0, dtype=torch.int64, device=device)
    draw = int(want * oversample)
    for rnd in range(6):
        deg = user_degrees(cfg.n_users, cfg.n_items, draw, cfg.alpha_user, seed + 7 * rnd)
        offs = np.zeros(cfg.n_users + 1, dtype=np.int64)
        np.cumsum(deg, out=offs[1:])
        E = int(offs[-1])
        offs_t = torch.from_numpy(offs).to(device)
        u = torch.empty(E, dtype=torch.int32, device=device)
        i = torch.empty(E, dtype=torch.int32, device=device)
        _lib.check(L.lgx_synth_edges(np.uint64(seed * 1_000_003 + rnd).item(), offs_t.data_ptr(), cfg.n_users,
                                     cdf_t.data_ptr(), perm_t.data_ptr(), cfg.n_items, E, u.data_ptr(), i.data_ptr(),
                                     _stream_ptr(device)), "lgx_synth_edges")
        new = u.to(torch.int64) * cfg.n_items + i.to(torch.int64)
        del u, i
        keys = torch.unique(torch.cat([keys, new]))
        del new
        if keys.numel() >= want:
            break
        draw = int((want - keys.numel()) * 1.5) + 1024
    if keys.numel() > want:  # deterministic trim: drop the pairs with the largest hash
        h = (keys * -7046029254386353131) ^ (keys >> 29)  # golden-ratio hash (0x9E3779B97F4A7C15 as int64)
        keep = torch.argsort(h)[:want]
        keys = torch.sort(keys[keep]).values
    users = (keys // cfg.n_items).to(torch.int32)
    items = (keys % cfg.n_items).to(torch.int32)
    return users, items


def synth_graph(cfg: GraphConfig, seed: int = 2020, device="cuda") -> CSRGraph:
    users, items = synth_edges(cfg, seed, device)
    return build_norm_adj(users, items, cfg.n_users, cfg.n_items, dedup=True, device=device)
