"""Evaluation drop-ins: the PyTorch ``Procedure.Test`` loop, the TF ``batch_test.test`` loop and
the C++ evaluator entry ``eval_score_matrix_foldout`` -- scoring, masking and top-k on the GPU.

References:
  Procedure.Test              lightGCN/LightGCN-PyTorch-master/code/Procedure.py:96-174
  test_one_batch / metrics    Procedure.py:60-72, code/utils.py:218-285
  batch_test.test             LightGCN-tf/utility/batch_test.py:25-84
  eval_score_matrix_foldout   LightGCN-tf/evaluator/cpp/evaluate_foldout.py:12-18
                              (-> apt_evaluate_foldout.pyx:22-65 -> tools.h + evaluate_foldout.h)
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Sequence

import numpy as np
import torch

from . import ops


def eval_score_matrix_foldout(score_matrix, test_items, top_k: int = 20, thread_num=None) -> np.ndarray:
    """Same signature/return as the reference: float32 [B, 5*top_k] = [pre|rec|ap|ndcg|mrr] curves.

    ``thread_num`` is accepted for signature compatibility (the GPU needs no host thread pool)."""
    if len(score_matrix) != len(test_items):
        raise ValueError("The lengths of score_matrix and test_items are not equal.")
    S = torch.as_tensor(np.ascontiguousarray(score_matrix, dtype=np.float32) if not torch.is_tensor(score_matrix)
                        else score_matrix)
    S = S.to(device="cuda", dtype=torch.float32).contiguous()
    idx, _ = ops.topk_rows(S, top_k)
    truth = ops.lists_to_device_csr(test_items, S.device, sort=False)
    return ops.foldout_metrics(idx, truth).cpu().numpy()


# --------------------------------------------------------------------------- PyTorch Test metrics
def _label(test_data: Sequence[Sequence[int]], pred: np.ndarray) -> np.ndarray:
    """utils.getLabel (code/utils.py:277-285): r[i, j] = 1.0 if pred[i, j] is in test_data[i].
    One sorted-key membership search for the whole batch instead of a set per user."""
    pred = np.asarray(pred, dtype=np.int64)
    n = len(test_data)
    if pred.ndim != 2 or pred.shape[0] != n:
        raise ValueError(f"pred must be [{n}, k]")
    lens = np.fromiter(map(len, test_data), dtype=np.int64, count=n)
    flat = np.fromiter(itertools.chain.from_iterable(test_data), dtype=np.int64, count=int(lens.sum()))
    if flat.size == 0 or pred.size == 0:
        return np.zeros(pred.shape, dtype=float)
    M = int(max(flat.max(), pred.max())) + 1
    keys = np.unique(np.repeat(np.arange(n, dtype=np.int64), lens) * M + flat)
    q = np.arange(n, dtype=np.int64)[:, None] * M + pred
    pos = np.minimum(np.searchsorted(keys, q), keys.size - 1)
    return ((keys[pos] == q) & (pred >= 0)).astype(float)


def test_one_batch(rating_k: np.ndarray, ground_true: Sequence[Sequence[int]], topks: Sequence[int]) -> Dict:
    """Procedure.test_one_batch (Procedure.py:60-72) with RecallPrecision_ATk / NDCGatK_r
    (code/utils.py:218-262), vectorised over users: the same float64 arrays as the reference's
    per-user loops, reduced in the same order, so the sums are identical."""
    recall_n = np.fromiter(map(len, ground_true), dtype=np.int64, count=len(ground_true))
    return _metrics(_label(ground_true, rating_k), recall_n, topks)


def _metrics_dev(hit: torch.Tensor, recall_n: torch.Tensor, topks: Sequence[int]) -> Dict:
    """_metrics on the device in float64: the same per-user terms (getLabel's 0 / 1, right / len,
    dcg / idcg with 1 / log2(j + 2)), summed over users by torch instead of numpy -- the sums agree to
    float64 rounding (the reference itself adds them batch by batch, Procedure.py:159-163)."""
    r = hit.to(torch.float64)
    n = recall_n.to(torch.float64)
    out = {"recall": [], "precision": [], "ndcg": []}
    for k in topks:
        right = r[:, :k].sum(1)
        out["recall"].append(torch.sum(right / n))
        out["precision"].append(torch.sum(right) / k)
        w = 1.0 / torch.log2(torch.arange(2, k + 2, device=r.device, dtype=torch.float64))
        tm = (torch.arange(k, device=r.device)[None, :] < torch.clamp(recall_n, max=k)[:, None]).to(torch.float64)
        idcg = torch.sum(tm * w, dim=1)
        dcg = torch.sum(r[:, :k] * w, dim=1)
        idcg[idcg == 0.] = 1.
        nd = dcg / idcg
        nd[torch.isnan(nd)] = 0.
        out["ndcg"].append(torch.sum(nd))
    return {key: torch.stack(v).cpu().numpy() for key, v in out.items()}


def _metrics(r: np.ndarray, recall_n: np.ndarray, topks: Sequence[int]) -> Dict:
    """RecallPrecision_ATk / NDCGatK_r sums over a batch from its hit matrix r (float64 0/1)."""
    pre, rec, ndcg = [], [], []
    for k in topks:
        right = r[:, :k].sum(1)
        rec.append(np.sum(right / recall_n))
        pre.append(np.sum(right) / k)
        tm = (np.arange(k)[None, :] < np.minimum(k, recall_n)[:, None]).astype(float)
        idcg = np.sum(tm * 1. / np.log2(np.arange(2, k + 2)), axis=1)
        dcg = np.sum(r[:, :k] * (1. / np.log2(np.arange(2, k + 2))), axis=1)
        idcg[idcg == 0.] = 1.
        nd = dcg / idcg
        nd[np.isnan(nd)] = 0.
        ndcg.append(np.sum(nd))
    return {"recall": np.array(rec), "precision": np.array(pre), "ndcg": np.array(ndcg)}


def _fingerprint(lists, keys) -> tuple:
    """A cheap content check of a dict / sequence of lists at a few fixed keys: (length, first, last)
    of each sampled list.  Catches a list edited in place (same dict object, same length) without
    walking the whole dict on every call."""
    out = []
    for u in keys:
        v = lists[u]
        n = len(v)
        out.append((n, int(v[0]) if n else -1, int(v[-1]) if n else -1))
    return tuple(out)


def _sample_keys(seq, n: int = 32) -> list:
    """Up to n evenly spaced entries of seq (always its first and last)."""
    if len(seq) <= n:
        return list(seq)
    return [seq[int(i)] for i in np.linspace(0, len(seq) - 1, n).round().astype(np.int64)]


def clear_caches() -> None:
    """Drop the device lists Test / batch_test keep between calls (and the dicts they hold).  Call it
    after changing testDict, train_items, test_set or a dataset's positives in a way the built-in
    check (same objects, same lengths, the same lists at 32 sampled users) cannot see, or to free
    the device memory once evaluation is over."""
    _TestLists._cache.clear()
    _BatchLists._cache.clear()


# Users whose mask holds more than dense_mask_min(n_items, d) items are ranked by the dense route
# (ops.score_topk_dense_masked) when the catalog is small enough for dense rows (the evaluation
# shapes): their 256-bit Bloom filter is saturated, so in the fused walk every one of their masked
# items that reaches the running threshold takes an exact search.  On propagated LightGCN tables a
# user's train items are among its best scores, and power-law users mask thousands of them
# (tools/mask_probe.py, profiles/r05_mask_probe.txt: the ~5 % of Gowalla-shape users above 64 masked
# items cost 1.6 ms of the 5.1 ms fused launch).  The dense route runs beside the fused launch
# (_Route.topk): while the fused walk leaves CUs idle -- fewer users than one round of its
# workgroups, 256 x 256 users at d <= 128 (8 waves x 32 users), 256 x 128 above -- dense rows cost
# nothing until they outlast it, and the threshold is the floor of 64 (profiles/r05_route_probe_side.txt:
# Amazon-book shape 14.70 ms at 357, 14.14 ms at 64; Gowalla flat from 64 to 128).  Otherwise a
# dense row adds its n_items * d to the call and the threshold grows with it (best near 64 at the
# Gowalla shape, 256-1024 at the Amazon-book shape when the two parts ran one after the other,
# profiles/r05_route_probe.txt).
DENSE_MASK_MIN = 64
DENSE_MAX_ITEMS = 1 << 18


def dense_mask_min(n_items: int, d: int, n_users: int = None) -> int:
    if n_users is not None and n_users <= 256 * (256 if d <= 128 else 128):
        return DENSE_MASK_MIN
    return max(DENSE_MASK_MIN, n_items * d // 32768)


_SIDE_STREAMS: Dict[str, torch.cuda.Stream] = {}


def _side_stream(dev) -> torch.cuda.Stream:
    key = str(torch.device(dev))
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=dev)
    return s


class _Route:
    """The split of an evaluation set between the fused launch and the dense route."""

    def __init__(self, rows: torch.Tensor, mask, n_items: int, k_max: int, d: int, thr: int = None,
                 chunk_bytes: int = None):
        self.rows, self.mask = rows, mask
        self.chunk_bytes = ops.DENSE_CHUNK_BYTES if chunk_bytes is None else int(chunk_bytes)
        n = rows.numel()
        lens = (mask[0][1:] - mask[0][:-1]) if mask is not None else None
        heavy = torch.zeros(n, dtype=torch.bool, device=rows.device)
        self.thr = dense_mask_min(n_items, d, n) if thr is None else thr
        if lens is not None and n_items <= DENSE_MAX_ITEMS:
            heavy = (lens > self.thr) & (lens <= n_items - k_max)
        self.n_heavy = int(heavy.sum())
        if self.n_heavy == 0:
            self.light_pos = None
            return
        self.light_pos = torch.nonzero(~heavy).flatten()
        self.heavy_pos = torch.nonzero(heavy).flatten()
        self.light_rows, self.heavy_rows = rows[self.light_pos].contiguous(), rows[self.heavy_pos].contiguous()
        self.light_mask = ops.csr_rows(mask, self.light_pos)
        self.heavy_mask = ops.csr_rows(mask, self.heavy_pos)
        step = ops.dense_chunk_users(n_items, self.chunk_bytes)
        self.heavy_offsets = [ops.dense_mask_offsets(self.heavy_mask, n_items, c0, min(self.n_heavy, c0 + step))
                              for c0 in range(0, self.n_heavy, step)]

    def topk(self, users: torch.Tensor, items: torch.Tensor, k: int, mask_value: float, apply_sigmoid: bool):
        """idx int32 [n, k] for every user of the set, in set order."""
        if self.light_pos is None:
            return ops.score_topk(users, items, k, user_rows=self.rows, mask=self.mask, mask_value=mask_value,
                                  apply_sigmoid=apply_sigmoid)[0]
        idx = torch.empty((self.rows.numel(), k), dtype=torch.int32, device=users.device)
        if not self.light_pos.numel():
            idx[self.heavy_pos] = ops.score_topk_dense_masked(users, items, k, self.heavy_rows, self.heavy_mask,
                                                              chunk_bytes=self.chunk_bytes, offsets=self.heavy_offsets)
            return idx
        # The dense route runs on a side stream beside the fused launch.  The fused walk holds one
        # workgroup per CU (its LDS) on ceil(users / users per workgroup) CUs -- 203 of 256 at the
        # Amazon-book shape, 208 at the Gowalla shape -- and the dense kernels take the rest.  The
        # side stream starts from the inputs' point on the caller's stream (before the fused launch)
        # and the caller's stream waits for it before the merge.
        main = torch.cuda.current_stream(users.device)
        side = _side_stream(users.device)
        # the score chunk (up to 1 GiB) comes from the caller's stream and is marked as used by the
        # side stream: freed, it returns to the caller's pool (training reuses it) once the side
        # stream's work is done, instead of staying reserved in the side stream's pool
        n_items = items.shape[0]
        scratch = torch.empty(min(self.n_heavy, ops.dense_chunk_users(n_items, self.chunk_bytes)) * n_items,
                              dtype=torch.float32, device=users.device)
        scratch.record_stream(side)
        side.wait_stream(main)
        light = ops.score_topk(users, items, k, user_rows=self.light_rows, mask=self.light_mask,
                               mask_value=mask_value, apply_sigmoid=apply_sigmoid)[0]
        with torch.cuda.stream(side):
            heavy = ops.score_topk_dense_masked(users, items, k, self.heavy_rows, self.heavy_mask,
                                                chunk_bytes=self.chunk_bytes, offsets=self.heavy_offsets,
                                                scratch=scratch)
        main.wait_stream(side)
        heavy.record_stream(main)
        del scratch
        idx[self.light_pos] = light
        idx[self.heavy_pos] = heavy
        return idx


class _TestLists:
    """The static lists of one evaluation set on the device: the test users (row ids), their train
    positives (the mask CSR) and their test items as sorted (row * M + item) keys.  Procedure.Test
    runs every few epochs over the same testDict / allPos; building these from Python lists was most
    of its time (profiles/r04_rows.json, a7 phases), so they are kept for as long as the same
    testDict object is passed (the reference never mutates it after loading, dataloader.py:282-293)
    and the lists of 32 sampled users, test items and positives, still read the same (_fingerprint);
    clear_caches() drops them."""

    _cache: Dict[tuple, "_TestLists"] = {}

    def __init__(self, dataset, testDict, n_items: int, dev):
        self.testDict = testDict  # held: its id cannot be reused while cached
        self.users = list(testDict.keys())
        n = len(self.users)
        self.rows = torch.as_tensor(self.users, dtype=torch.int64, device=dev)
        self.mask = ops.lists_to_device_csr(dataset.getUserPosItems(self.users), dev, sort=True)
        self.probe = _sample_keys(self.users)
        self.stamp = self.fingerprint(dataset)
        self.routes: Dict[tuple, _Route] = {}
        truths = [testDict[u] for u in self.users]
        self.recall_n = np.fromiter(map(len, truths), dtype=np.int64, count=n)
        self.recall_n_dev = torch.from_numpy(self.recall_n).to(dev)
        flat = np.fromiter(itertools.chain.from_iterable(truths), dtype=np.int64, count=int(self.recall_n.sum()))
        self.M = int(max(n_items, int(flat.max()) + 1 if flat.size else 0, 1))
        keys = np.repeat(np.arange(n, dtype=np.int64), self.recall_n) * self.M + flat
        self.keys = torch.unique(torch.from_numpy(keys).to(dev))  # sorted
        # the same lists as a CSR (sorted, deduplicated) for lgx_test_metrics
        bounds = torch.arange(n + 1, device=dev, dtype=torch.int64) * self.M
        self.truth = (torch.searchsorted(self.keys, bounds), (self.keys % self.M).to(torch.int32))

    def route(self, n_items: int, k: int, d: int) -> _Route:
        key = (n_items, k, d)
        if key not in self.routes:
            self.routes[key] = _Route(self.rows, self.mask, n_items, k, d)
        return self.routes[key]

    def fingerprint(self, dataset) -> tuple:
        try:
            return (_fingerprint(self.testDict, self.probe),
                    _fingerprint(list(dataset.getUserPosItems(self.probe)), range(len(self.probe))))
        except (KeyError, IndexError):
            return ()

    @classmethod
    def get(cls, dataset, n_items: int, dev) -> "_TestLists":
        td = dataset.testDict
        key = (id(dataset), id(td), len(td), n_items, str(dev))
        hit = cls._cache.get(key)
        if hit is None or hit.testDict is not td or hit.fingerprint(dataset) != hit.stamp:
            cls._cache.clear()
            hit = cls._cache[key] = cls(dataset, td, n_items, dev)
        return hit

    def hit_mask(self, idx: torch.Tensor) -> torch.Tensor:
        """utils.getLabel on the device: bool [n, k], True where idx[i, j] is a test item of user i."""
        if self.keys.numel() == 0:
            return torch.zeros(tuple(idx.shape), dtype=torch.bool, device=idx.device)
        q = torch.arange(idx.shape[0], device=idx.device, dtype=torch.int64)[:, None] * self.M + idx.long()
        pos = torch.searchsorted(self.keys, q.reshape(-1)).clamp_(max=self.keys.numel() - 1).view_as(q)
        return (self.keys[pos] == q) & (idx >= 0)

    def hits(self, idx: torch.Tensor) -> np.ndarray:
        """The hit matrix as getLabel returns it (float64 0 / 1, on the host)."""
        return self.hit_mask(idx).to(torch.uint8).cpu().numpy().astype(float)


def Test(dataset, Recmodel, epoch=0, w=None, multicore=0, topks: Sequence[int] = (20,)) -> Dict:
    """Procedure.Test on the fused engine: one propagation, one fused score+mask+top-k launch for
    all test users (sigmoid scores, positives set to -(1<<10) as Procedure.py:134), and one launch
    for the hits and the float64 metric sums (lgx_test_metrics)."""
    Recmodel = Recmodel.eval()
    max_K = max(topks)
    results = {"precision": np.zeros(len(topks)), "recall": np.zeros(len(topks)), "ndcg": np.zeros(len(topks))}
    with torch.no_grad():
        all_users, all_items = Recmodel.computer()
        tl = _TestLists.get(dataset, all_items.shape[0], all_users.device)
        idx = tl.route(all_items.shape[0], max_K, all_items.shape[1]).topk(all_users, all_items, max_K,
                                                                          -float(1 << 10), True)
        # getLabel + RecallPrecision_ATk + NDCGatK_r for every user in one launch (lgx_test_metrics)
        sums = ops.test_metrics(idx, tl.truth, topks, tl.recall_n_dev).cpu().numpy()
        res = {"recall": sums[0], "precision": sums[1] / np.asarray(topks, dtype=np.float64), "ndcg": sums[2]}
        for key in results:
            results[key] = res[key] / float(len(tl.users))
    return results


# --------------------------------------------------------------------------- TF batch_test
class _BatchLists:
    """batch_test's per-user lists on the device: row ids, the train-item mask (flag 0) and the
    truth lists, built once for a given (users, train_items, test_set, flag) and reused while the
    same dict objects and the same users (every one compared) come back (the reference's
    data_generator holds them for the whole run, batch_test.py:12-23) and the train / test lists of
    32 sampled users still read the same; clear_caches() drops them."""

    _cache: Dict[tuple, "_BatchLists"] = {}

    def __init__(self, users_to_test, users: np.ndarray, train_items, test_set, flag: int, dev):
        self.train_items, self.test_set, self.users = train_items, test_set, users  # held (ids stay valid)
        # a shallow snapshot of the caller's list: comparing it with the list again is a pointer walk
        # while the entries are the same int objects (~50 us at 50 K users), and a value compare only
        # where an entry was replaced -- every user is checked on every call
        self.users_snap = list(users_to_test) if isinstance(users_to_test, list) else None
        ul = users.tolist()
        self.probe = _sample_keys(ul)
        self.stamp = self.fingerprint()
        self.rows = torch.as_tensor(users, dtype=torch.int64, device=dev)
        if flag == 0:
            truths = [test_set[u] for u in ul]
            self.mask = ops.lists_to_device_csr([train_items[u] for u in ul], dev, sort=True)  # KeyError as :64
        else:
            truths = [train_items[u] for u in ul]
            self.mask = None
        # sorted (the fold-out curves treat a truth list as a set; lgx_foldout_metrics binary-searches
        # long sorted lists)
        self.truth = ops.lists_to_device_csr(truths, dev, sort=True)
        self.routes: Dict[tuple, _Route] = {}

    def route(self, n_items: int, k: int, d: int) -> _Route:
        key = (n_items, k, d)
        if key not in self.routes:
            self.routes[key] = _Route(self.rows, self.mask, n_items, k, d)
        return self.routes[key]

    def fingerprint(self) -> tuple:
        try:
            return (_fingerprint(self.train_items, self.probe),
                    _fingerprint(self.test_set, self.probe) if self.test_set is not None else ())
        except (KeyError, IndexError, TypeError):
            return ()

    @classmethod
    def get(cls, users_to_test, train_items, test_set, flag: int, dev) -> "_BatchLists":
        key = (id(train_items), id(test_set), len(users_to_test), flag, str(dev))
        hit = cls._cache.get(key)
        if hit is not None and hit.train_items is train_items and hit.test_set is test_set:
            # the same users, all of them: the reference passes data_generator's list every time
            # (batch_test.py:12-23), compared against the snapshot; any other sequence by value
            if hit.users_snap is not None and isinstance(users_to_test, list):
                same = users_to_test == hit.users_snap
            elif isinstance(users_to_test, np.ndarray):
                same = users_to_test.shape == hit.users.shape and np.array_equal(users_to_test, hit.users)
            else:
                same = np.array_equal(hit.users, np.fromiter((int(u) for u in users_to_test), dtype=np.int64))
            if same and hit.fingerprint() == hit.stamp:
                return hit
        users = np.fromiter((int(u) for u in users_to_test), dtype=np.int64)
        cls._cache.clear()
        hit = cls._cache[key] = cls(users_to_test, users, train_items, test_set, flag, dev)
        return hit


def batch_test(user_emb: torch.Tensor, item_emb: torch.Tensor, users_to_test: Sequence[int],
               train_items: Dict[int, Sequence[int]], test_set: Dict[int, Sequence[int]],
               Ks: Sequence[int] = (20,), train_set_flag: int = 0) -> Dict:
    """batch_test.test (batch_test.py:25-84): raw dot-product ratings, training items set to -inf
    and the test set as truth (train_set_flag=0, :57-65), or no mask and the train items as truth
    (train_set_flag=1, :66-68); top-max(Ks), fold-out curves, and their mean over users as the
    reference's np.mean(all_result, axis=0) computes it (:75-76: float32 sums in user order, one float32
    division), on the device bit for bit (lgx_column_mean_f32)."""
    top_show = np.sort(np.asarray(Ks))
    max_top = int(max(top_show))
    bl = _BatchLists.get(users_to_test, train_items, test_set, train_set_flag, user_emb.device)
    idx = bl.route(item_emb.shape[0], max_top, item_emb.shape[1]).topk(user_emb, item_emb, max_top,
                                                                       float("-inf"), False)
    curves = ops.foldout_metrics(idx, bl.truth)
    # the users' mean on the device: only 5 x max_top values cross to the host
    mean = ops.column_mean(curves).cpu().numpy()
    final = mean.reshape(5, max_top)[:, top_show - 1].reshape(5, len(top_show))
    return {"precision": final[0].astype(np.float64), "recall": final[1].astype(np.float64),
            "ndcg": final[3].astype(np.float64)}
