"""BPR sampling on the GPU.

Drop-ins for the reference's cppimport extension ``sources/sampling.cpp`` (``seed``,
``sample_negative``, ``sample_negative_ByUser``, :27-86, :88-100) and for
``utils.UniformSample_original`` (code/utils.py:55-64).  Rows are drawn by ``lgx_sample_bpr``:
[user, one of the user's positives, neg_num items that are not positives].

The reference draws with libc ``rand()`` seeded from the clock, so the rows match its distribution,
not its bits.  Here every call takes the next seed of a counter-based stream started by ``seed()``
(deterministic across runs for a given seed).  Users with no positive produce no row (the C++
indexes an empty vector there; the Python fallback skips them, utils.py:84-85).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .ops import _stream_ptr, lists_to_device_csr, require_gpu

_state = {"seed": 2020, "calls": 0}  # parse.py:43's default seed


def seed(s: int) -> None:
    """sampling.seed / set_seed: restart the draw stream."""
    _state["seed"] = int(s)
    _state["calls"] = 0


def _next_seed() -> int:
    _state["calls"] += 1
    x = (_state["seed"] * 0x9E3779B97F4A7C15 + _state["calls"]) & 0xFFFFFFFFFFFFFFFF
    return x


def sample_device(pos: Tuple[torch.Tensor, torch.Tensor], n_items: int, per_user: Optional[int] = None,
                  users: Optional[torch.Tensor] = None, neg_num: int = 1, seed_value: Optional[int] = None,
                  drop_invalid: bool = True) -> torch.Tensor:
    """``lgx_sample_bpr`` on device-resident positives (indptr int64 [U+1], items int32, each user's
    items sorted).  Either per_user rows for every user, or one row per entry of ``users``.
    Returns int32 [rows, 2 + neg_num] on the device."""
    indptr, items = pos
    require_gpu(indptr, items, users)
    n_users = indptr.shape[0] - 1
    if users is not None:
        users = users.to(torch.int32).contiguous()
        n_rows = users.shape[0]
        per = 0
    else:
        if not per_user or per_user <= 0:
            raise ValueError("per_user must be > 0 when no user list is given")
        n_rows, per = n_users * per_user, per_user
    out = torch.empty((max(n_rows, 1), 2 + neg_num), dtype=torch.int32, device=indptr.device)
    s = _next_seed() if seed_value is None else int(seed_value)
    _lib.check(_lib.lib().lgx_sample_bpr(indptr.data_ptr(), items.data_ptr(), n_users, int(n_items),
                                         users.data_ptr() if users is not None else None, n_rows, per, neg_num,
                                         s, out.data_ptr(), _stream_ptr(indptr.device)),
               "lgx_sample_bpr")
    out = out[:n_rows]
    if drop_invalid:
        out = out[(out[:, 1:] >= 0).all(dim=1)]
    return out


def _positives(allPos: Sequence[Sequence[int]], device) -> Tuple[torch.Tensor, torch.Tensor]:
    return lists_to_device_csr(allPos, device, sort=True)


def sample_negative(user_num: int, item_num: int, train_num: int, allPos, neg_num: int,
                    device="cuda") -> np.ndarray:
    """sources/sampling.cpp:27-56: train_num // user_num rows per user -> int32 [rows, neg_num + 2]."""
    per = max(1, train_num // max(1, user_num))
    pos = _positives(allPos.select(range(user_num)) if hasattr(allPos, "select") else list(allPos)[:user_num],
                     device)
    return sample_device(pos, item_num, per_user=per, neg_num=neg_num).cpu().numpy()


def sample_negative_ByUser(users, item_num: int, allPos, neg_num: int, device="cuda") -> np.ndarray:
    """sources/sampling.cpp:58-86: one row per listed user -> int32 [len(users), neg_num + 2]."""
    pos = _positives(allPos if hasattr(allPos, "device_csr") else list(allPos), device)
    u = torch.as_tensor(np.asarray(users, dtype=np.int32), device=device)
    return sample_device(pos, item_num, users=u, neg_num=neg_num).cpu().numpy()


def UniformSample_original(dataset, neg_ratio: int = 1, device="cuda") -> np.ndarray:
    """utils.UniformSample_original (code/utils.py:55-64) with the GPU sampler."""
    return sample_negative(dataset.n_users, dataset.m_items, dataset.trainDataSize, dataset.allPos, neg_ratio,
                           device=device)
