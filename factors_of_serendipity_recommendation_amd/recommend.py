"""recommend.py similarity drop-ins on the GPU (rows a11 / a12 of SURVEY.md section 8).

  accuracy_cf          recommend.py:208-223 (+ sub_argpartition :53-56): per user, dot products of
                       E_u with the user's ~1000 candidate items, top-K -> data/<ds>/rec/<seed>/rec_acc.npy
  similarity_minmax    recommend.py:163-164 (elasticity_item) and :375-377 (stratification):
                       global min / max of E_user . E_item^T, computed inside the fused scoring
                       kernel without materialising the [U, I] matrix

Same signatures and side effects as the reference.  The per-user work runs in lgx_gather_scores +
lgx_topk_rows instead of a Python loop feeding a multiprocessing.Pool.  The reference's
np.argpartition returns the top-K as an unordered set; this module returns it ordered by
descending score (ties -> earlier candidate position), which is one of the orders argpartition
may produce.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from . import ops


def candidate_scores(emb_user: torch.Tensor, emb_item: torch.Tensor,
                     candidates: Sequence[Sequence[int]]) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Ragged per-user candidate dots -> (scores f32 [n_pairs], indptr int64 [U+1], items int32)."""
    dev = emb_user.device
    indptr, items = ops.lists_to_device_csr(candidates, dev, sort=False)
    n_pairs = int(indptr[-1].item())
    return ops.gather_scores(emb_user, emb_item, (indptr, items), n_pairs), indptr, items


def topk_candidates(emb_user: torch.Tensor, emb_item: torch.Tensor, candidates: Sequence[Sequence[int]],
                    K: int = 20) -> np.ndarray:
    """For each user the K candidate items with the largest <E_u, E_i> -> int64 [U, K]."""
    scores, indptr, items = candidate_scores(emb_user, emb_item, candidates)
    U = len(candidates)
    lens = torch.diff(indptr)
    width = int(lens.max().item()) if U else 0
    if width < K:
        raise ValueError(f"every user needs at least K={K} candidates")
    # pack the ragged scores into a padded [U, width] matrix (-inf padding never wins)
    dense = torch.full((U, width), float("-inf"), dtype=torch.float32, device=scores.device)
    rows = torch.repeat_interleave(torch.arange(U, device=scores.device), lens)
    cols = torch.arange(scores.numel(), device=scores.device) - indptr[:-1][rows]
    dense[rows, cols] = scores
    pos, _ = ops.topk_rows(dense, K)
    picked = items.long()[indptr[:-1, None] + pos.long()]
    return picked.cpu().numpy().astype(np.int64)


def accuracy_cf(mat_candidate: Dict[int, List[int]], dataset_name: str, seed: int, K: int = 20,
                data_root: str = "data", device="cuda") -> None:
    """recommend.accuracy_cf: same inputs (data/<ds>/emb_{item,user}.npy, candidate dict), same
    output file data/<ds>/rec/<seed>/rec_acc.npy of shape [U, K]."""
    emb_item = np.load(os.path.join(data_root, dataset_name, "emb_item.npy"), allow_pickle=False)
    emb_user = np.load(os.path.join(data_root, dataset_name, "emb_user.npy"), allow_pickle=False)
    eu = torch.from_numpy(np.ascontiguousarray(emb_user, dtype=np.float32)).to(device)
    ei = torch.from_numpy(np.ascontiguousarray(emb_item, dtype=np.float32)).to(device)
    cands = [mat_candidate[u] for u in range(len(mat_candidate))]
    mat_rec = topk_candidates(eu, ei, cands, K)
    out_dir = os.path.join(data_root, dataset_name, "rec", str(seed))
    os.makedirs(out_dir, exist_ok=True)
    np.save(os.path.join(out_dir, "rec_acc.npy"), mat_rec)


def similarity_minmax(emb_user: torch.Tensor, emb_item: torch.Tensor) -> Tuple[float, float]:
    """(min, max) of emb_user . emb_item^T over all pairs (recommend.py:163-164)."""
    _, _, mm = ops.score_topk(emb_user.contiguous(), emb_item.contiguous(), 1, want_minmax=True)
    mm = mm.cpu().numpy()
    return float(mm[0]), float(mm[1])
