"""recommend.py similarity drop-ins on the GPU (rows a11 / a12 and 8(f) rank 1 of SURVEY.md).

  accuracy_cf          recommend.py:208-223 (+ sub_argpartition :53-56): per user, dot products of
                       E_u with the user's ~1000 candidate items, top-K -> data/<ds>/rec/<seed>/rec_acc.npy
  similarity_minmax    recommend.py:163-164 (elasticity_item) and :375-377 (stratification):
                       global min / max of E_user . E_item^T, computed inside the fused scoring
                       kernel without materialising the [U, I] matrix
  difference           recommend.py:287-312: per candidate, max dot with the user's train items
                       (lgx_list_dot_reduce), scaled by the item . item^T min / max -> rec_dif.npy
  elasticity_item      recommend.py:149-205 (+ :144-145): scaled user-candidate dot plus the user's
                       elasticity; the K candidates closest to alpha * mean -> rec_ela.npy

Same signatures and side effects as the reference.  The per-user work runs in lgx_gather_scores +
lgx_topk_rows instead of a Python loop feeding a multiprocessing.Pool.  The reference's
np.argpartition returns the top-K as an unordered set; this module returns it ordered by
descending score (ties -> earlier candidate position), which is one of the orders argpartition
may produce.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

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


def ragged_topk(scores: torch.Tensor, indptr: torch.Tensor, items: torch.Tensor, K: int) -> np.ndarray:
    """Per user, the K list entries with the largest f32 score (descending, ties -> earlier position):
    the ragged scores are packed into a -inf padded [U, width] matrix for lgx_topk_rows."""
    U = indptr.shape[0] - 1
    lens = torch.diff(indptr)
    width = int(lens.max().item()) if U else 0
    shortest = int(lens.min().item()) if U else 0
    if U and shortest < K:
        # np.argpartition(score, -K) raises on a list shorter than K (recommend.py:53-56); never
        # return -inf padding positions, which would index the next user's candidates
        raise ValueError(f"every user needs at least K={K} candidates (shortest list has {shortest})")
    dense = torch.full((U, width), float("-inf"), dtype=torch.float32, device=scores.device)
    rows = torch.repeat_interleave(torch.arange(U, device=scores.device), lens)
    cols = torch.arange(scores.numel(), device=scores.device) - indptr[:-1][rows]
    dense[rows, cols] = scores
    pos, _ = ops.topk_rows(dense, K)
    picked = items.long()[indptr[:-1, None] + pos.long()]
    return picked.cpu().numpy().astype(np.int64)


def topk_candidates(emb_user: torch.Tensor, emb_item: torch.Tensor, candidates: Sequence[Sequence[int]],
                    K: int = 20) -> np.ndarray:
    """For each user the K candidate items with the largest <E_u, E_i> -> int64 [U, K]."""
    scores, indptr, items = candidate_scores(emb_user, emb_item, candidates)
    return ragged_topk(scores, indptr, items, K)


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


def item_dot_minmax(emb_item: torch.Tensor) -> Tuple[float, float]:
    """(min, max) of emb_item . emb_item^T (recommend.py:291-292; utils.py:500-529's blocked loop)."""
    return similarity_minmax(emb_item, emb_item)


def train_lists(dataset_name: str, n_users: int, data_root: str = "data") -> List[List[int]]:
    """rating_train.csv grouped by userInd, the i-th group for user i (the reference zips the groups
    with range(len(mat_candidate)), recommend.py:297-298)."""
    import pandas as pd
    df = pd.read_csv(os.path.join(data_root, dataset_name, "rating_train.csv"), usecols=["userInd", "itemInd"])
    groups = [g["itemInd"].values.tolist() for _, g in df.groupby("userInd")]
    return groups[:n_users]


def difference_scores(emb_item: torch.Tensor, candidates: Sequence[Sequence[int]],
                      history: Sequence[Sequence[int]]) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """diffscore = 1 - (max_t <E_c, E_t> - min_dis) / (max_dis - min_dis) per candidate c of each user,
    max over the user's history t (recommend.py:305-307)."""
    dev = emb_item.device
    a = ops.lists_to_device_csr(candidates, dev, sort=False)
    b = ops.lists_to_device_csr(history, dev, sort=False)
    m = ops.list_dot_reduce(emb_item, a, b, "max")
    mn, mx = item_dot_minmax(emb_item)
    return 1.0 - (m - mn) / (mx - mn), a[0], a[1]


def difference(mat_candidate: Dict[int, List[int]], dataset_name: str, seed: int, K: int = 20,
               data_root: str = "data", device="cuda") -> None:
    """recommend.difference: same inputs (emb_item.npy, rating_train.csv, candidates), same output
    data/<ds>/rec/<seed>/rec_dif.npy [U, K] (the top-K set by diffscore, here ordered)."""
    emb_item = np.load(os.path.join(data_root, dataset_name, "emb_item.npy"), allow_pickle=False)
    ei = torch.from_numpy(np.ascontiguousarray(emb_item, dtype=np.float32)).to(device)
    cands = [mat_candidate[u] for u in range(len(mat_candidate))]
    scores, indptr, items = difference_scores(ei, cands, train_lists(dataset_name, len(cands), data_root))
    out_dir = os.path.join(data_root, dataset_name, "rec", str(seed))
    os.makedirs(out_dir, exist_ok=True)
    np.save(os.path.join(out_dir, "rec_dif.npy"), ragged_topk(scores, indptr, items, K))


def elasticity_keys(emb_user: torch.Tensor, emb_item: torch.Tensor, candidates: Sequence[Sequence[int]],
                    num_item: np.ndarray, alpha: float = 1.0) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """-|factor - alpha * mean(factor)| per candidate (larger = closer), factor = scaled user-candidate
    dot + the user's min-max scaled item count (recommend.py:162-185); float64 as in the reference."""
    scores, indptr, items = candidate_scores(emb_user, emb_item, candidates)
    mn, mx = similarity_minmax(emb_user, emb_item)
    cnt = torch.as_tensor(np.asarray(num_item, dtype=np.float64), device=scores.device)
    ela = (cnt - cnt.min()) / (cnt.max() - cnt.min())
    lens = torch.diff(indptr)
    rows = torch.repeat_interleave(torch.arange(len(candidates), device=scores.device), lens)
    factor = (scores.double() - mn) / (mx - mn) + ela[rows]
    key = -(factor - alpha * factor.mean()).abs()
    return key.float(), indptr, items


def elasticity_item(mat_candidate: Dict[int, List[int]], dataset_name: str, seed: int, K: int = 20,
                    alpha: float = 1.0, data_root: str = "data", device="cuda", **kwargs) -> None:
    """recommend.elasticity_item: same inputs (user.csv num_item, emb_{user,item}.npy, candidates),
    same output data/<ds>/rec/<seed>/rec_ela.npy [U, K] (the K candidates with the smallest
    |factor - alpha * mean|, here ordered by that distance)."""
    import pandas as pd
    df_user = pd.read_csv(os.path.join(data_root, dataset_name, "user.csv"))
    emb_item = np.load(os.path.join(data_root, dataset_name, "emb_item.npy"), allow_pickle=False)
    emb_user = np.load(os.path.join(data_root, dataset_name, "emb_user.npy"), allow_pickle=False)
    eu = torch.from_numpy(np.ascontiguousarray(emb_user, dtype=np.float32)).to(device)
    ei = torch.from_numpy(np.ascontiguousarray(emb_item, dtype=np.float32)).to(device)
    cands = [mat_candidate[u] for u in range(len(mat_candidate))]
    key, indptr, items = elasticity_keys(eu, ei, cands, df_user["num_item"].values, alpha)
    out_dir = os.path.join(data_root, dataset_name, "rec", str(seed))
    os.makedirs(out_dir, exist_ok=True)
    np.save(os.path.join(out_dir, "rec_ela.npy"), ragged_topk(key, indptr, items, K))


def stratification_bounds(emb_user: torch.Tensor, emb_item: torch.Tensor, num_fold: int = 10,
                          epsilon: float = 0.1) -> Tuple[float, float]:
    """(min_dis, inter) of recommend.py:375-378 in numpy's float16 arithmetic.  The float16 cast is
    monotone, so the extremes of the cast matrix are the casts of the fp32 extremes (fused kernel)."""
    mn, mx = similarity_minmax(emb_user, emb_item)
    max_dis, min_dis = np.float16(mx) + epsilon, np.float16(mn)
    inter = (max_dis - min_dis) / num_fold
    return float(min_dis), float(inter)


def fused_labels_eligible(emb_user: torch.Tensor, d: int) -> bool:
    """lgx_strat_labels_fused covers 5..32 MFMA chunks per row (f32 d 40..256, bf16 d 80..256)."""
    per = 8 if emb_user.dtype == torch.float32 else 16
    return emb_user.dtype in (torch.float32, torch.bfloat16) and d % (per // 2) == 0 and 4 * per < d <= 256


def strat_labels(emb_user: torch.Tensor, emb_item: torch.Tensor, mask_indptr: torch.Tensor,
                 mask_indices: torch.Tensor, min16: float, inter16: float, num_fold: int,
                 fused: Optional[bool] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Labels [U, I] int8 and label counts [U, num_fold + 1] of recommend.py:375-381 for a batch of
    users: fused (the MFMA epilogue labels the scores; no [U, I] f32 matrix) when the shape allows,
    else lgx_score_dense rows + lgx_strat_labels.  Both give the same bits."""
    from . import _lib
    dev = emb_user.device
    U, I = emb_user.shape[0], emb_item.shape[0]
    L = _lib.lib()
    st = ops._stream_ptr(dev)
    labels = torch.empty((U, I), dtype=torch.int8, device=dev)
    hist = torch.empty((U, num_fold + 1), dtype=torch.int32, device=dev)
    if fused is None:
        fused = fused_labels_eligible(emb_user, emb_user.shape[1])
    if fused:
        Q, it = emb_user.contiguous(), emb_item.contiguous()
        _lib.check(L.lgx_strat_labels_fused(Q.data_ptr(), None, it.data_ptr(), U, I, Q.shape[1], ops._dtype_code(Q),
                                            min16, inter16, num_fold, mask_indptr.data_ptr(), mask_indices.data_ptr(),
                                            labels.data_ptr(), hist.data_ptr(), st), "lgx_strat_labels_fused")
    else:
        S = ops.score_dense(emb_user.contiguous(), emb_item)
        _lib.check(L.lgx_strat_labels(S.data_ptr(), U, I, min16, inter16, num_fold, mask_indptr.data_ptr(),
                                      mask_indices.data_ptr(), labels.data_ptr(), hist.data_ptr(), st),
                   "lgx_strat_labels")
        del S
    return labels, hist


def stratified_candidates(emb_user: torch.Tensor, emb_item: torch.Tensor, train: Sequence[Sequence[int]],
                          targets: Sequence[int], num_fold: int = 10, epsilon: float = 0.1, seed: int = 0,
                          batch: int = 4096, fused: Optional[bool] = None) -> List[List[int]]:
    """Per user, the stratified candidate list of create_candidates_stratification_sub +
    sample_list (recommend.py:314-356): labels and counts by strat_labels (fused into the scoring
    kernel's epilogue where the shape allows), the per-label random picks by lgx_strat_select."""
    from . import _lib
    dev = emb_user.device
    U, I = emb_user.shape[0], emb_item.shape[0]
    min16, inter16 = stratification_bounds(emb_user, emb_item, num_fold, epsilon)
    mp, mi = ops.lists_to_device_csr(train, dev, sort=True)
    tgt = torch.as_tensor(np.asarray(targets, dtype=np.int32), device=dev)
    K = int(max(1, int(tgt.max().item()) if U else 1))
    out_lists: List[List[int]] = []
    L = _lib.lib()
    st = ops._stream_ptr(dev)
    pin = dev.type == "cuda"

    def unpack(p):
        # the host's list building for batch b runs while the GPU labels and selects batch b+1
        ev, o_h, c_h = p
        ev.synchronize()
        o, c = o_h.numpy(), c_h.numpy()
        rows = o.tolist()  # one C call for the whole batch; only short rows get trimmed
        for j in np.flatnonzero(c < o.shape[1]).tolist():
            rows[j] = rows[j][:c[j]]
        out_lists.extend(rows)

    pending = None
    for b0 in range(0, U, batch):
        b1 = min(U, b0 + batch)
        labels, hist = strat_labels(emb_user[b0:b1], emb_item, mp[b0:], mi, min16, inter16, num_fold, fused)
        out = torch.empty((b1 - b0, K), dtype=torch.int32, device=dev)
        cnt = torch.empty(b1 - b0, dtype=torch.int32, device=dev)
        _lib.check(L.lgx_strat_select(labels.data_ptr(), b1 - b0, I, hist.data_ptr(), num_fold + 1,
                                      tgt[b0:b1].contiguous().data_ptr(), (seed * 0x9E3779B97F4A7C15 + b0) % 2 ** 64,
                                      out.data_ptr(), K, cnt.data_ptr(), st), "lgx_strat_select")
        o_h = torch.empty(out.shape, dtype=torch.int32, pin_memory=pin)
        c_h = torch.empty(cnt.shape, dtype=torch.int32, pin_memory=pin)
        o_h.copy_(out, non_blocking=pin)
        c_h.copy_(cnt, non_blocking=pin)
        ev = torch.cuda.Event() if pin else None
        if ev is not None:
            ev.record()
        if pending is not None:
            unpack(pending)
        pending = (ev if ev is not None else _Done(), o_h, c_h)
    if pending is not None:
        unpack(pending)
    return out_lists


class _Done:
    """Event stand-in for a batch whose copies already completed (synchronous, non-CUDA device)."""

    def synchronize(self) -> None:
        pass


def create_candidates_stratification(dataset_name: str, seed: int, K_c: int = 1000, num_fold: int = 10,
                                     epsilon: float = 0.1, data_root: str = "data", device="cuda") -> Dict[int, List[int]]:
    """recommend.create_candidates_stratification: per user the stratified sample of K_c - |test|
    non-train items followed by the user's test items; saved as rec/<seed>/candidate.npy (a pickled
    dict, as np.save writes it) and returned.  The cache files are not read back (always recomputed)."""
    import pandas as pd
    emb_item = np.load(os.path.join(data_root, dataset_name, "emb_item.npy"), allow_pickle=False)
    emb_user = np.load(os.path.join(data_root, dataset_name, "emb_user.npy"), allow_pickle=False)
    eu = torch.from_numpy(np.ascontiguousarray(emb_user, dtype=np.float32)).to(device)
    ei = torch.from_numpy(np.ascontiguousarray(emb_item, dtype=np.float32)).to(device)
    U = eu.shape[0]
    train = train_lists(dataset_name, U, data_root)
    test = pd.read_csv(os.path.join(data_root, dataset_name, "rating_test.csv")) \
        .groupby("userInd")["itemInd"].apply(list).to_dict()
    targets = [K_c - len(test.get(u, [])) for u in range(len(train))]
    cands = stratified_candidates(eu[:len(train)], ei, train, targets, num_fold, epsilon, seed)
    mat_candidate = {u: c + list(test.get(u, [])) for u, c in enumerate(cands)}
    out_dir = os.path.join(data_root, dataset_name, "rec", str(seed))
    os.makedirs(out_dir, exist_ok=True)
    np.save(os.path.join(out_dir, "candidate.npy"), mat_candidate)
    return mat_candidate
