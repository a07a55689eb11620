"""CPU baseline: the reference's own CPU execution of the hot path, restated with the same library
calls it makes (torch.sparse.mm / torch.matmul / torch.topk on the host).

TEST / BENCH INFRASTRUCTURE ONLY -- imported by bench.py's ``cpu_baseline`` leg and tests, never
by the product package.  ``kind = "port"`` in the bench JSON.

  propagate_cpu   LightGCN.computer()          lightGCN/LightGCN-PyTorch-master/code/model.py:149-176
                  (torch.sparse.mm x K, stack, mean, split)
  score_topk_cpu  getUsersRating + Test mask   model.py:179-184, Procedure.py:127-135
"""
from __future__ import annotations

import time

import numpy as np
import torch


def coo_from_csr(indptr: np.ndarray, indices: np.ndarray, vals: np.ndarray, n_cols: int) -> torch.Tensor:
    """Coalesced float32 sparse COO (dataloader.py:331-337, 373-374)."""
    rows = np.repeat(np.arange(len(indptr) - 1, dtype=np.int64), np.diff(indptr))
    idx = torch.from_numpy(np.stack([rows, indices.astype(np.int64)]))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(vals.astype(np.float32)),
                                   (len(indptr) - 1, n_cols)).coalesce()


def propagate_cpu(G: torch.Tensor, all_emb: torch.Tensor, K: int) -> torch.Tensor:
    """model.py:153-175 on the host."""
    embs = [all_emb]
    for _ in range(K):
        all_emb = torch.sparse.mm(G, all_emb)
        embs.append(all_emb)
    return torch.mean(torch.stack(embs, dim=1), dim=1)


def time_spmm_rows(G_block: torch.Tensor, X: torch.Tensor, K: int, threads: int) -> dict:
    """Time K x torch.sparse.mm(G_block, X) (one row block of A^ against the full table)."""
    torch.set_num_threads(threads)
    torch.sparse.mm(G_block, X)  # warm-up
    t0 = time.perf_counter()
    for _ in range(K):
        torch.sparse.mm(G_block, X)
    t = time.perf_counter() - t0
    nnz = G_block._nnz()
    return {"seconds": t, "edges": K * nnz, "edges_per_s": K * nnz / t, "threads": threads}


def score_topk_cpu(Q: torch.Tensor, items: torch.Tensor, k: int, masks=None, batch: int = 100) -> tuple:
    """Procedure.py:121-135 per 100-user batch: matmul + sigmoid + -(1<<10) mask + torch.topk."""
    out = []
    t0 = time.perf_counter()
    for s in range(0, Q.shape[0], batch):
        rating = torch.sigmoid(torch.matmul(Q[s:s + batch], items.t()))
        if masks is not None:
            for r, m in enumerate(masks[s:s + batch]):
                rating[r, torch.as_tensor(m, dtype=torch.long)] = -(1 << 10)
        out.append(torch.topk(rating, k=k)[1])
    t = time.perf_counter() - t0
    return torch.cat(out), t
