"""utils.py serendipity metrics on the GPU.

  ser1_sub / ser1   utils.py:23-66    acc = scaled max dot of each recommended item with the user's
                                      test items, dif = 1 - scaled max dot with the train items,
                                      ser = harmonic mean of the two
  ser2_sub / ser2   utils.py:117-141  mean over the recommended items outside the user's pm row of
                                      the max dot with the train items, scaled
  diversity         utils.py:265-287  1 - scaled mean of each list's pairwise dot matrix
  item_dot_minmax   utils.py:500-529  the blocked min / max of emb_item . emb_item^T that scales them

Every per-user numpy product of the reference is one ``lgx_list_dot_reduce`` launch over all users;
the global min / max comes from the fused scoring kernel (items as queries), never materialising
the [I, I] matrix.  Inputs are the reference's files (emb_item.npy, rating_{train,test}.csv,
rec/<seed>/pm.npy); the same (dataset_name, mat_rec, max_dis, min_dis[, seed]) signatures.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import ops
from .recommend import item_dot_minmax  # noqa: F401  (re-exported: utils.evaluate's min / max)


def _grouped(dataset_name: str, name: str, data_root: str) -> List[List[int]]:
    import pandas as pd
    df = pd.read_csv(os.path.join(data_root, dataset_name, name), usecols=["userInd", "itemInd"])
    return [g["itemInd"].values.tolist() for _, g in df.groupby("userInd")]


def _emb_item(dataset_name: str, data_root: str, device) -> torch.Tensor:
    e = np.load(os.path.join(data_root, dataset_name, "emb_item.npy"), allow_pickle=False)
    return torch.from_numpy(np.ascontiguousarray(e, dtype=np.float32)).to(device)


def list_max_dot(emb_item: torch.Tensor, lists_a: Sequence[Sequence[int]],
                 lists_b: Sequence[Sequence[int]]) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per user, max over B(u) of <E_a, E_b> for each a in A(u) -> (values f32 [nnz(A)], indptr)."""
    dev = emb_item.device
    a = ops.lists_to_device_csr(lists_a, dev, sort=False)
    b = ops.lists_to_device_csr(lists_b, dev, sort=False)
    return ops.list_dot_reduce(emb_item, a, b, "max"), a[0]


def ser1_batch(emb_item: torch.Tensor, mat_rec: np.ndarray, train: Sequence[Sequence[int]],
               test: Sequence[Sequence[int]], max_dis: float, min_dis: float):
    """ser1_sub for every user at once: (mean acc, mean dif, mean ser, acc [U, K], dif [U, K])."""
    recs = [np.asarray(r).astype(int).tolist() for r in mat_rec]
    U, K = len(recs), len(recs[0]) if recs else 0
    mt, _ = list_max_dot(emb_item, recs, test)
    mr, _ = list_max_dot(emb_item, recs, train)
    acc = ((mt.double() - min_dis) / (max_dis - min_dis)).view(U, K)
    dif = (1 - (mr.double() - min_dis) / (max_dis - min_dis)).view(U, K)
    ser = 2 * acc * dif / (acc + dif)
    return (float(acc.mean(1).mean()), float(dif.mean(1).mean()), float(ser.mean(1).mean()),
            acc.cpu().numpy(), dif.cpu().numpy())


def ser1(dataset_name: str, mat_rec: np.ndarray, max_dis: float, min_dis: float, data_root: str = "data",
         device="cuda"):
    """utils.ser1: the balance between accuracy and difference; same return tuple."""
    train = _grouped(dataset_name, "rating_train.csv", data_root)
    test = _grouped(dataset_name, "rating_test.csv", data_root)
    n = min(len(train), len(test), len(mat_rec))  # the reference zips the three
    return ser1_batch(_emb_item(dataset_name, data_root, device), np.asarray(mat_rec)[:n], train[:n], test[:n],
                      max_dis, min_dis)


def ser2_batch(emb_item: torch.Tensor, mat_rec: np.ndarray, mat_pm: np.ndarray, train: Sequence[Sequence[int]],
               max_dis: float, min_dis: float) -> float:
    """ser2 over all users: per user the mean over rec \\ pm of the max dot with the train items
    (min_dis when rec \\ pm is empty), averaged and scaled."""
    rest = [sorted(set(np.asarray(r).tolist()) - set(np.asarray(p).tolist())) for r, p in zip(mat_rec, mat_pm)]
    m, indptr = list_max_dot(emb_item, rest, train)
    lens = torch.diff(indptr)
    rows = torch.repeat_interleave(torch.arange(len(rest), device=m.device), lens)
    sums = torch.zeros(len(rest), dtype=torch.float64, device=m.device).index_add_(0, rows, m.double())
    per_user = torch.where(lens > 0, sums / lens.clamp(min=1).double(),
                           torch.full_like(sums, float(min_dis)))
    return (float(per_user.mean()) - min_dis) / (max_dis - min_dis)


def ser2(dataset_name: str, mat_rec: np.ndarray, max_dis: float, min_dis: float, seed, data_root: str = "data",
         device="cuda") -> float:
    """utils.ser2: same inputs (rating_train.csv, rec/<seed>/pm.npy), same scalar."""
    train = _grouped(dataset_name, "rating_train.csv", data_root)
    mat_pm = np.load(os.path.join(data_root, dataset_name, "rec", str(seed), "pm.npy"), allow_pickle=False)
    n = min(len(train), len(mat_rec), len(mat_pm))
    return ser2_batch(_emb_item(dataset_name, data_root, device), np.asarray(mat_rec)[:n], mat_pm[:n], train[:n],
                      max_dis, min_dis)


def diversity_batch(emb_item: torch.Tensor, mat_rec: np.ndarray, max_dis: float, min_dis: float) -> float:
    """diversity_sub for every user: 1 - (mean of E_rec E_rec^T - min_dis) / (max_dis - min_dis), averaged."""
    recs = [np.asarray(r).astype(int).tolist() for r in mat_rec]
    dev = emb_item.device
    a = ops.lists_to_device_csr(recs, dev, sort=False)
    s = ops.list_dot_reduce(emb_item, a, a, "sum").double()
    lens = torch.diff(a[0])
    rows = torch.repeat_interleave(torch.arange(len(recs), device=dev), lens)
    tot = torch.zeros(len(recs), dtype=torch.float64, device=dev).index_add_(0, rows, s)
    mean = tot / (lens.double() ** 2)
    return float((1 - (mean - min_dis) / (max_dis - min_dis)).mean())


def diversity(dataset_name: str, mat_rec: np.ndarray, max_dis: float, min_dis: float, data_root: str = "data",
              device="cuda") -> float:
    """utils.diversity: same inputs, same scalar."""
    return diversity_batch(_emb_item(dataset_name, data_root, device), mat_rec, max_dis, min_dis)
