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
from collections.abc import Mapping, Sequence
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import ops

# pinned staging slots of stratified_candidates' per-batch device-to-host copies
_STAGE = 3


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
    mm = ops.score_minmax(emb_user, emb_item).cpu().numpy()
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


def legacy_float16_bounds(max16: float, min16: float, num_fold: int, epsilon: float) -> Tuple[float, float]:
    """(min_dis, inter) of recommend.py:377-381 under the numpy the reference pins (1.19.5,
    environment.yml:253; 1.22.3 at :140), i.e. legacy value-based promotion, not NEP 50:
      np.max(mat_dis) + epsilon   float16 scalar + Python float -> float64
      (max_dis - min_dis) / num_fold                             -> float64
      (mat_dis - min_dis) / inter  float16 array / float64 scalar -> float16 loop: inter is
                                   rounded to float16 once, here.
    numpy >= 2 (NEP 50) would round max_dis and inter to float16 step by step instead and move
    every label boundary by an ulp for about a third of (max, min) pairs."""
    mx16, mn16 = np.float16(max16), np.float16(min16)
    inter = (float(mx16) + float(epsilon) - float(mn16)) / num_fold   # float64, as numpy 1.x
    return float(mn16), float(np.float16(inter))


def stratification_bounds(emb_user: torch.Tensor, emb_item: torch.Tensor, num_fold: int = 10,
                          epsilon: float = 0.1) -> Tuple[float, float]:
    """(min_dis, inter16) of recommend.py:375-381.  The float16 cast is monotone, so the extremes
    of the cast matrix are the casts of the fp32 extremes (computed inside the fused kernel)."""
    mn, mx = similarity_minmax(emb_user, emb_item)
    return legacy_float16_bounds(mx, mn, num_fold, epsilon)


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
    ops.require_gpu(emb_user, emb_item, mask_indptr, mask_indices)
    ops.check_pair(emb_user, emb_item)
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


class CandidateLists(Sequence):
    """The candidate lists of a stratified_candidates call: row u is picks[u, :counts[u]] of the flat
    int32 output the GPU wrote, turned into a Python list only when it is read.  Compares equal to
    a list of lists with the same rows; pickles as a plain list of lists (what the reference
    pickles to list_res.pickle, recommend.py:434-435)."""

    def __init__(self, picks: np.ndarray, counts: np.ndarray):
        self.picks, self.counts = picks, counts

    def __len__(self) -> int:
        return len(self.counts)

    def row(self, u: int) -> np.ndarray:
        return self.picks[u, :self.counts[u]]

    def __getitem__(self, u):
        if isinstance(u, slice):
            return [self[j] for j in range(*u.indices(len(self)))]
        return self.row(u).tolist()

    def __iter__(self):
        return (self.row(u).tolist() for u in range(len(self)))

    def __eq__(self, other) -> bool:
        if isinstance(other, CandidateLists):
            return len(self) == len(other) and np.array_equal(self.counts, other.counts) and all(
                np.array_equal(self.row(u), other.row(u)) for u in range(len(self)))
        try:
            return len(self) == len(other) and all(a == b for a, b in zip(self, other))
        except TypeError:
            return NotImplemented

    def __reduce__(self):
        return (list, (), None, iter(self))


def stratified_candidates(emb_user: torch.Tensor, emb_item: torch.Tensor, train, targets: Sequence[int],
                          num_fold: int = 10, epsilon: float = 0.1, seed: int = 0, batch: int = 4096,
                          fused: Optional[bool] = None,
                          bounds: Optional[Tuple[float, float]] = None) -> CandidateLists:
    """Per user, the stratified candidate list of create_candidates_stratification_sub +
    sample_list (recommend.py:314-356): labels and counts by strat_labels (fused into the scoring
    kernel's epilogue where the shape allows), the per-label random picks by lgx_strat_select.

    ``train`` is a list of per-user train item lists, or a (indptr, indices) CSR pair.  Raises
    ValueError where the reference's sampling raises: a negative target (DataFrame.sample(n < 0))
    or a list that sample_list cannot pad to its target (random.sample(lst, k > len(lst)),
    recommend.py:317).  ``bounds`` = (min_dis, inter16) when the label grid comes from more users
    than are labelled here (the reference's np.max / np.min run over the whole emb_user @ emb_item.T,
    recommend.py:375-377); by default they come from emb_user itself.  Each batch's picks go through
    a small ring of pinned staging buffers into one pageable host array, the copy of batch b
    overlapping the GPU work of the next batches; rows become lists only when read
    (CandidateLists)."""
    from . import _lib
    dev = torch.device(emb_user.device)
    ops.require_gpu(emb_user, emb_item)
    ops.check_pair(emb_user, emb_item)
    U, I = emb_user.shape[0], emb_item.shape[0]
    tgt_h = np.asarray(targets, dtype=np.int64)
    if tgt_h.shape != (U,):
        raise ValueError(f"targets must have one entry per user ({U}), got shape {tgt_h.shape}")
    if U and tgt_h.min() < 0:
        raise ValueError(f"negative candidate target {int(tgt_h.min())} (more test items than K_c)")
    if U and tgt_h.max() > 1024:
        raise ValueError("at most 1024 candidates per user")
    with torch.cuda.device(dev):
        if bounds is None:
            min16, inter16 = stratification_bounds(emb_user, emb_item, num_fold, epsilon)
        else:
            min16, inter16 = (float(x) for x in bounds)
        if isinstance(train, tuple):
            mp, mi = (t.to(dev) for t in train)
            mi = mi.to(torch.int32)
        else:
            mp, mi = ops.lists_to_device_csr(train, dev, sort=True)
        if mp.numel() != U + 1:
            raise ValueError(f"train has {mp.numel() - 1} users, emb_user {U}")
        tgt = torch.as_tensor(tgt_h.astype(np.int32), device=dev)
        K = int(max(1, int(tgt_h.max()) if U else 1))
        L = _lib.lib()
        stream = torch.cuda.current_stream(dev)
        st = ops._stream_ptr(dev)
        picks = np.empty((U, K), dtype=np.int32)
        counts = np.empty(U, dtype=np.int32)
        # pinned staging: a ring of _STAGE batch slots (not U x K pinned bytes: 4 GB at 1 M users x
        # 1000 candidates, slow to page-lock); slot j is drained into the pageable arrays once the
        # copy that last filled it has completed
        nring = min(_STAGE, -(-U // batch)) if U else 0
        ring = [(torch.empty((batch, K), dtype=torch.int32, pin_memory=True),
                 torch.empty(batch, dtype=torch.int32, pin_memory=True)) for _ in range(nring)]
        pending = [None] * nring  # (event, b0, b1) of the copy in flight into each slot

        def drain(j):
            ev, c0, c1 = pending[j]
            ev.synchronize()
            picks[c0:c1] = ring[j][0][:c1 - c0].numpy()
            counts[c0:c1] = ring[j][1][:c1 - c0].numpy()
            pending[j] = None

        for bi, b0 in enumerate(range(0, U, batch)):
            b1 = min(U, b0 + batch)
            labels, hist = strat_labels(emb_user[b0:b1], emb_item, mp[b0:], mi, min16, inter16, num_fold, fused)
            out = torch.empty((b1 - b0, K), dtype=torch.int32, device=dev)
            cnt = torch.empty(b1 - b0, dtype=torch.int32, device=dev)
            _lib.check(L.lgx_strat_select(labels.data_ptr(), b1 - b0, I, hist.data_ptr(), num_fold + 1,
                                          tgt[b0:b1].contiguous().data_ptr(),
                                          (seed * 0x9E3779B97F4A7C15 + b0) % 2 ** 64,
                                          out.data_ptr(), K, cnt.data_ptr(), st), "lgx_strat_select")
            # async D2H on the stream the kernels ran on: the copy engine drains batch b while the
            # next batch's labels run (the allocator keeps `out` alive until the copy is done)
            j = bi % nring
            if pending[j] is not None:
                drain(j)
            ring[j][0][:b1 - b0].copy_(out, non_blocking=True)
            ring[j][1][:b1 - b0].copy_(cnt, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            pending[j] = (ev, b0, b1)
        for j in range(nring):
            if pending[j] is not None:
                drain(j)
    res = CandidateLists(picks, counts)
    short = np.flatnonzero(res.counts < tgt_h)
    if short.size:
        u = int(short[0])
        raise ValueError(f"user {u}: {int(res.counts[u])} of {int(tgt_h[u])} candidates -- sample_list cannot pad "
                         f"(random.sample: sample larger than population, recommend.py:317)")
    return res


def train_csr(dataset_name: str, n_users: int, data_root: str = "data") -> Tuple[torch.Tensor, torch.Tensor]:
    """rating_train.csv as a sorted, de-duplicated CSR: row j = the j-th userInd group, as the
    reference zips mat_label with df_train.groupby("userInd") (recommend.py:372,421-422)."""
    indptr, items, _ = train_groups(dataset_name, n_users, data_root)
    return indptr, items


def train_groups(dataset_name: str, n_users: int, data_root: str = "data"):
    """train_csr plus the group keys: users[j] = the userInd of group j (sorted, groupby order),
    the ``uind`` the reference pairs with row j of mat_label (recommend.py:421)."""
    import pandas as pd
    df = pd.read_csv(os.path.join(data_root, dataset_name, "rating_train.csv"), usecols=["userInd", "itemInd"])
    u = df["userInd"].to_numpy(np.int64)
    it = df["itemInd"].to_numpy(np.int64)
    key = np.unique((u << 32) | it)                 # sorted by (user, item), duplicates dropped
    ku = key >> 32
    users, lens = np.unique(ku, return_counts=True)  # groups in groupby order
    lens = lens[:n_users]
    indptr = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=indptr[1:])
    items = (key[:indptr[-1]] & 0xFFFFFFFF).astype(np.int32)
    return torch.from_numpy(indptr), torch.from_numpy(items), users[:len(lens)]


class CandidateDict(Mapping):
    """create_candidates_stratification's {user: candidates + test items} (recommend.py:444-451)
    over the flat GPU output: a user's list is built on first access and then kept (so in-place
    edits of it persist, as with the reference's dict); pickles (np.save) as a plain dict."""

    def __init__(self, lists: Sequence[Sequence[int]], tests: Sequence[Sequence[int]]):
        self._lists, self._tests, self._memo = lists, tests, {}

    def __len__(self) -> int:
        return len(self._lists)

    def __iter__(self):
        return iter(range(len(self._lists)))

    def __contains__(self, u) -> bool:
        return isinstance(u, (int, np.integer)) and 0 <= u < len(self._lists)

    def __getitem__(self, u):
        if u not in self:
            raise KeyError(u)
        u = int(u)
        got = self._memo.get(u)
        if got is None:
            got = self._memo[u] = list(self._lists[u]) + list(self._tests[u])
        return got

    def __reduce__(self):
        return (dict, (), None, None, iter(self.items()))


def _save_object(path: str, obj) -> None:
    """np.save(path, obj) as the reference calls it on a dict: a 0-d object array, pickled."""
    arr = np.empty((), dtype=object)
    arr[()] = obj
    np.save(path, arr)


def create_candidates_stratification(dataset_name: str, seed: int, K_c: int = 1000, num_fold: int = 10,
                                     epsilon: float = 0.1, data_root: str = "data", device="cuda"):
    """recommend.create_candidates_stratification (recommend.py:359-452): per user the stratified
    sample of K_c - |test| non-train items followed by the user's test items.

    The reference's caches are honoured as it honours them: rec/<seed>/candidate.npy is returned
    when it holds one entry per user (:365-368); rec/<seed>/list_res.pickle, when present, replaces
    the sampling (:436-440) and is written after it (:434-435).  Both are files this function
    (or the reference) wrote, read back with pickle as the reference reads them.  A user without
    test items raises KeyError (:426); targets the sampling cannot meet raise ValueError
    (stratified_candidates).  Returns a CandidateDict (a lazy Mapping over the flat picks) and
    writes candidate.npy as the reference's plain dict."""
    import pickle
    import pandas as pd
    out_dir = os.path.join(data_root, dataset_name, "rec", str(seed))
    path_candidate = os.path.join(out_dir, "candidate.npy")
    path_list_res = os.path.join(out_dir, "list_res.pickle")
    emb_item = np.load(os.path.join(data_root, dataset_name, "emb_item.npy"), allow_pickle=False)
    emb_user = np.load(os.path.join(data_root, dataset_name, "emb_user.npy"), allow_pickle=False)
    if os.path.exists(path_candidate):
        mat_candidate = np.load(path_candidate, allow_pickle=True).item()
        if emb_user.shape[0] == len(mat_candidate):
            return mat_candidate
    test = pd.read_csv(os.path.join(data_root, dataset_name, "rating_test.csv")) \
        .groupby("userInd")["itemInd"].apply(list).to_dict()
    if not os.path.exists(path_list_res):
        indptr, items, uinds = train_groups(dataset_name, emb_user.shape[0], data_root)
        n = indptr.numel() - 1
        # zip(mat_label, group_train): row j of the labels (user j) with the j-th group, whose key
        # uind picks the test list that sets the target (recommend.py:421,426)
        targets = [K_c - len(test[int(u)]) for u in uinds]           # KeyError as at :426
        eu = torch.from_numpy(np.ascontiguousarray(emb_user, dtype=np.float32)).to(device)
        ei = torch.from_numpy(np.ascontiguousarray(emb_item, dtype=np.float32)).to(device)
        # the label grid spans the whole emb_user @ emb_item.T (recommend.py:375-377), also when
        # fewer train groups than users are labelled
        bounds = stratification_bounds(eu, ei, num_fold, epsilon)
        list_res = stratified_candidates(eu[:n], ei, (indptr, items), targets, num_fold, epsilon, seed,
                                         bounds=bounds)
        os.makedirs(out_dir, exist_ok=True)
        with open(path_list_res, "wb") as f:
            pickle.dump(list_res, f)
    else:
        with open(path_list_res, "rb") as f:
            list_res = pickle.load(f)
    tests = [test[u] for u in range(len(list_res))]                 # KeyError as at :450
    mat_candidate = CandidateDict(list_res, tests)
    os.makedirs(out_dir, exist_ok=True)
    _save_object(path_candidate, mat_candidate)
    return mat_candidate
