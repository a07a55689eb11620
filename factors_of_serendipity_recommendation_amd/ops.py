"""Tensor-level wrappers over the liblgx C ABI (all GPU, stream-ordered on torch's current stream).

Every function validates shapes/devices on the host, allocates outputs + workspace through torch's
caching allocator and calls exactly one C entry point; no computation happens in Python and there
is no CPU path.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional, Sequence, Tuple

import torch

from . import _lib
from .graph import CSRGraph, _stream_ptr, require_gpu

_DT = {torch.float32: _lib.LGX_DTYPE_F32, torch.bfloat16: _lib.LGX_DTYPE_BF16}


def _dtype_code(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported embedding dtype {t.dtype}; use float32 or bfloat16") from None


def _ptr(t: Optional[torch.Tensor]):
    return t.data_ptr() if t is not None else None


# ------------------------------------------------------------------------------------ propagation
def propagate_layer(A: CSRGraph, X: torch.Tensor, mode: int, Y: Optional[torch.Tensor] = None,
                    E0: Optional[torch.Tensor] = None, acc: Optional[torch.Tensor] = None,
                    out: Optional[torch.Tensor] = None, n_mean: float = 1.0) -> None:
    """One LightGCN layer (``lgx_propagate_layer``), writing into caller-provided buffers."""
    require_gpu(X)
    d = X.shape[1]
    cs = A.c_struct(d, X.element_size())
    _lib.check(_lib.lib().lgx_propagate_layer(ctypes.byref(cs), _ptr(X), _ptr(Y), _ptr(E0), _ptr(acc), _ptr(out),
                                              d, _dtype_code(X), mode, float(n_mean), _stream_ptr(X.device)),
               "lgx_propagate_layer")


def propagate_layer_stack(A: CSRGraph, X: torch.Tensor, E0: torch.Tensor, prev: Sequence[torch.Tensor],
                          out: torch.Tensor, n_mean: float) -> None:
    """The last layer over kept layer tables (``lgx_propagate_layer_stack``):
    out = (E0 + prev[0] + ... + prev[-1] + A X) / n_mean."""
    require_gpu(X, E0, out, *prev)
    d = X.shape[1]
    cs = A.c_struct(d, X.element_size())
    arr = (ctypes.c_void_p * max(1, len(prev)))(*[p.data_ptr() for p in prev])
    _lib.check(_lib.lib().lgx_propagate_layer_stack(ctypes.byref(cs), _ptr(X), _ptr(E0), arr, len(prev), _ptr(out),
                                                    d, _dtype_code(X), float(n_mean), _stream_ptr(X.device)),
               "lgx_propagate_layer_stack")


def layer_epilogue(y: torch.Tensor, mode: int, Y: Optional[torch.Tensor] = None, E0: Optional[torch.Tensor] = None,
                   acc: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, n_mean: float = 1.0,
                   dtype: Optional[torch.dtype] = None) -> None:
    """``lgx_layer_epilogue``: the layer epilogue of ``propagate_layer`` applied to precomputed fp32
    row sums ``y`` [rows, d] (the cross-rank sum of PARTIAL outputs).  ``dtype`` is the storage
    type of Y / E0 (default: Y's, else E0's, else float32)."""
    require_gpu(y)
    if y.dtype != torch.float32 or not y.is_contiguous():
        raise ValueError("y must be a contiguous float32 tensor")
    ref = Y if Y is not None else E0
    dt = dtype or (ref.dtype if ref is not None else torch.float32)
    code = _lib.LGX_DTYPE_BF16 if dt == torch.bfloat16 else _lib.LGX_DTYPE_F32
    _lib.check(_lib.lib().lgx_layer_epilogue(_ptr(y), y.shape[0], _ptr(Y), _ptr(E0), _ptr(acc), _ptr(out),
                                             y.shape[1], code, mode, float(n_mean), _stream_ptr(y.device)),
               "lgx_layer_epilogue")


def sum_slabs(src: torch.Tensor, out: torch.Tensor) -> None:
    """``lgx_sum_slabs``: out = src[0] + src[1] + ... + src[n-1], added in slab order in fp32
    (src [n, rows, d] and out [rows, d], contiguous float32): the deterministic reduce step of the
    sharded layer (distributed.py)."""
    require_gpu(src, out)
    if src.dtype != torch.float32 or out.dtype != torch.float32 or not (src.is_contiguous() and out.is_contiguous()):
        raise ValueError("sum_slabs: contiguous float32 tensors")
    if src.dim() < 2 or tuple(src.shape[1:]) != tuple(out.shape):
        raise ValueError(f"sum_slabs: src {tuple(src.shape)} vs out {tuple(out.shape)}")
    _lib.check(_lib.lib().lgx_sum_slabs(_ptr(src), src.shape[0], out.numel(), _ptr(out), _stream_ptr(out.device)),
               "lgx_sum_slabs")


def spmm(A: CSRGraph, X: torch.Tensor) -> torch.Tensor:
    """Y = A X (the reference's ``torch.sparse.mm(G, all_emb)``, model.py:171)."""
    require_gpu(X)
    X = X.contiguous()
    if X.shape[0] != A.n_cols:
        raise ValueError(f"X has {X.shape[0]} rows, operator has {A.n_cols} columns")
    Y = torch.empty((A.n_rows, X.shape[1]), dtype=X.dtype, device=X.device)
    cs = A.c_struct(X.shape[1], X.element_size())
    _lib.check(_lib.lib().lgx_spmm_csr(ctypes.byref(cs), X.data_ptr(), Y.data_ptr(), X.shape[1], _dtype_code(X),
                                       _stream_ptr(X.device)), "lgx_spmm_csr")
    return Y


def propagate(A: CSRGraph, E0: torch.Tensor, K: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """LightGCN.computer() body (model.py:149-175): mean over [E0, A E0, ..., A^K E0] -> fp32 [N, d].

    E0 may be float32 or bfloat16 (bf16 storage, fp32 accumulation)."""
    require_gpu(E0)
    E0 = E0.contiguous()
    N, d = E0.shape
    if N != A.n_rows or A.n_rows != A.n_cols:
        raise ValueError("propagate needs a square operator matching E0")
    if out is None:
        out = torch.empty((N, d), dtype=torch.float32, device=E0.device)
    L = _lib.lib()
    dt = _dtype_code(E0)
    ws = ctypes.c_size_t(0)
    _lib.check(L.lgx_propagate_workspace(N, d, dt, ctypes.byref(ws)), "lgx_propagate_workspace")
    work = torch.empty(max(ws.value, 1), dtype=torch.uint8, device=E0.device)
    cs = A.c_struct(d, E0.element_size())
    _lib.check(L.lgx_propagate(ctypes.byref(cs), E0.data_ptr(), out.data_ptr(), d, int(K), dt, work.data_ptr(),
                               ws.value, _stream_ptr(E0.device)), "lgx_propagate")
    return out


# ------------------------------------------------------------------------------------ scoring
def check_pair(Q: torch.Tensor, items: torch.Tensor) -> None:
    """Query rows and item rows of one scoring launch: same dtype and the same d (the kernels read
    both with one row stride)."""
    if Q.dtype != items.dtype:
        raise TypeError("Q and items must share a dtype")
    if Q.dim() != 2 or items.dim() != 2 or Q.shape[1] != items.shape[1]:
        raise ValueError(f"Q {tuple(Q.shape)} and items {tuple(items.shape)} must be [*, d] with one d")


def score_dense(Q: torch.Tensor, items: torch.Tensor, user_rows: Optional[torch.Tensor] = None,
                apply_sigmoid: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[B, I] scores (getUsersRating, model.py:179-184 / TF batch_ratings, LightGCN.py:148); out: an
    optional contiguous f32 [B, I] destination."""
    require_gpu(Q, items, user_rows)
    check_pair(Q, items)
    Q = Q.contiguous()
    items = items.contiguous()
    B = user_rows.numel() if user_rows is not None else Q.shape[0]
    rows = user_rows.to(torch.int64).contiguous() if user_rows is not None else None
    if out is None:
        out = torch.empty((B, items.shape[0]), dtype=torch.float32, device=Q.device)
    elif (out.dtype != torch.float32 or tuple(out.shape) != (B, items.shape[0]) or not out.is_contiguous()
          or out.device != Q.device):
        raise ValueError(f"score_dense: out must be a contiguous float32 [{B}, {items.shape[0]}] on {Q.device}")
    _lib.check(_lib.lib().lgx_score_dense(Q.data_ptr(), _ptr(rows), items.data_ptr(), B, items.shape[0], Q.shape[1],
                                          _dtype_code(Q), int(apply_sigmoid), out.data_ptr(),
                                          _stream_ptr(Q.device)), "lgx_score_dense")
    return out


def lists_to_device_csr(lists: Sequence[Sequence[int]], device, sort: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """Ragged python lists -> (indptr int64 [n+1], indices int32) on the device.  A
    ``dataloader.PosLists`` (already sorted and de-duplicated) is packed on the device directly."""
    import itertools
    import numpy as np
    if hasattr(lists, "device_csr"):
        ip, ix = lists.device_csr(device)
        return ip, ix.to(torch.int32)
    lens = np.fromiter(map(len, lists), dtype=np.int64, count=len(lists))
    indptr = np.zeros(len(lists) + 1, dtype=np.int64)
    np.cumsum(lens, out=indptr[1:])
    total = int(indptr[-1])
    if not total:
        return torch.from_numpy(indptr).to(device), torch.zeros(1, dtype=torch.int32, device=device)
    # one flat pass over the Python ints (no per-list array), the per-row sort as one sort of
    # (row << 32 | item) keys on the device
    flat = np.fromiter(itertools.chain.from_iterable(lists), dtype=np.int64, count=total)
    if not sort:
        return torch.from_numpy(indptr).to(device), torch.from_numpy(flat.astype(np.int32)).to(device)
    if flat.min() < 0 or flat.max() >= 2 ** 31:
        raise ValueError("list entries must be in [0, 2^31)")
    rows = np.repeat(np.arange(len(lists), dtype=np.int64), lens)
    key = torch.from_numpy((rows << 32) | flat).to(device)
    key = torch.sort(key).values
    return torch.from_numpy(indptr).to(device), (key & 0xFFFFFFFF).to(torch.int32)


def parse_lines(text: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """``lgx_parse_lines_*`` on a device uint8 tensor of "uid item item ..." text ->
    (line_user int32 [L], line_ptr int64 [L+1], items int32 [P], pair_user int32 [P])."""
    require_gpu(text)
    if text.dtype != torch.uint8 or not text.is_contiguous():
        raise ValueError("text must be a contiguous uint8 tensor")
    L = _lib.lib()
    n, dev, st = text.numel(), text.device, _stream_ptr(text.device)
    wsb = ctypes.c_size_t()
    _lib.check(L.lgx_parse_lines_workspace(n, ctypes.byref(wsb)), "lgx_parse_lines_workspace")
    ws = torch.empty(max(wsb.value, 1), dtype=torch.uint8, device=dev)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    _lib.check(L.lgx_parse_lines_count(text.data_ptr(), n, ws.data_ptr(), wsb.value, counts.data_ptr(), st),
               "lgx_parse_lines_count")
    n_numbers, n_lines = (int(x) for x in counts.tolist())
    n_pairs = n_numbers - n_lines
    line_user = torch.empty(max(n_lines, 1), dtype=torch.int32, device=dev)
    line_ptr = torch.empty(n_lines + 1, dtype=torch.int64, device=dev)
    items = torch.empty(max(n_pairs, 1), dtype=torch.int32, device=dev)
    pair_user = torch.empty(max(n_pairs, 1), dtype=torch.int32, device=dev)
    _lib.check(L.lgx_parse_lines_fill(text.data_ptr(), n, ws.data_ptr(), wsb.value, n_numbers, n_lines,
                                      line_user.data_ptr(), line_ptr.data_ptr(), items.data_ptr(),
                                      pair_user.data_ptr(), st), "lgx_parse_lines_fill")
    return line_user[:n_lines], line_ptr, items[:n_pairs], pair_user[:n_pairs]


def read_interactions_device(path: str, device="cuda"):
    """A LightGCN txt file parsed on the device (one host->device copy of its bytes)."""
    import numpy as np
    data = np.fromfile(path, dtype=np.uint8)
    return parse_lines(torch.from_numpy(data).to(device))


def list_dot_reduce(table: torch.Tensor, a_csr: Tuple[torch.Tensor, torch.Tensor],
                    b_csr: Tuple[torch.Tensor, torch.Tensor], reduce: str = "max") -> torch.Tensor:
    """``lgx_list_dot_reduce``: per user u, for each a in A(u) the max (or sum) over b in B(u) of
    <table[a], table[b]>.  a_csr / b_csr = (indptr int64 [U+1], items int32) on the device (same U).
    Returns f32 [nnz(A)] in A's order (-inf / 0 for an empty B(u))."""
    require_gpu(table)
    (ap, ai), (bp, bi) = a_csr, b_csr
    if ap.shape != bp.shape:
        raise ValueError("A and B must list the same users")
    table = table.contiguous()
    n_users = ap.shape[0] - 1
    n = int(ap[-1].item()) if n_users > 0 else 0
    out = torch.empty(max(n, 1), dtype=torch.float32, device=table.device)
    red = _lib.LGX_REDUCE_MAX if reduce == "max" else _lib.LGX_REDUCE_SUM
    _lib.check(_lib.lib().lgx_list_dot_reduce(table.data_ptr(), table.shape[1], _dtype_code(table), n_users,
                                              ap.data_ptr(), ai.data_ptr(), bp.data_ptr(), bi.data_ptr(), red,
                                              out.data_ptr(), _stream_ptr(table.device)), "lgx_list_dot_reduce")
    return out[:n]


def score_topk(Q: torch.Tensor, items: torch.Tensor, k: int, user_rows: Optional[torch.Tensor] = None,
               mask: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, mask_value: float = float("-inf"),
               apply_sigmoid: bool = False, want_minmax: bool = False):
    """Fused full-catalog score + positive mask + top-k (``lgx_score_topk``).

    mask = (indptr int64 [B+1], indices int32) with each row's excluded items SORTED ascending.
    Returns (idx int32 [B,k], val f32 [B,k]) or (idx, val, minmax f32[2])."""
    require_gpu(Q, items, user_rows)
    check_pair(Q, items)
    Q = Q.contiguous()
    items = items.contiguous()
    B = user_rows.numel() if user_rows is not None else Q.shape[0]
    rows = user_rows.to(torch.int64).contiguous() if user_rows is not None else None
    dev = Q.device
    idx = torch.empty((B, k), dtype=torch.int32, device=dev)
    val = torch.empty((B, k), dtype=torch.float32, device=dev)
    mm = torch.empty(2, dtype=torch.float32, device=dev) if want_minmax else None
    L = _lib.lib()
    ws = ctypes.c_size_t(0)
    _lib.check(L.lgx_score_topk_workspace(B, items.shape[0], k, ctypes.byref(ws)), "lgx_score_topk_workspace")
    work = torch.empty(max(ws.value, 1), dtype=torch.uint8, device=dev)
    mi, mx = (mask[0].contiguous(), mask[1].contiguous()) if mask is not None else (None, None)
    if mi is not None and mi.numel() != B + 1:
        raise ValueError("mask indptr must have B+1 entries")
    _lib.check(L.lgx_score_topk(Q.data_ptr(), _ptr(rows), items.data_ptr(), B, items.shape[0], Q.shape[1],
                                _dtype_code(Q), _ptr(mi), _ptr(mx), int(k), float(mask_value), int(apply_sigmoid),
                                idx.data_ptr(), val.data_ptr(), _ptr(mm), work.data_ptr(), ws.value,
                                _stream_ptr(dev)), "lgx_score_topk")
    return (idx, val, mm) if want_minmax else (idx, val)


def csr_rows(csr: Tuple[torch.Tensor, torch.Tensor], sel: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rows `sel` (int64, device) of a device CSR (indptr int64, indices), in that order."""
    ip, ix = csr
    lens = (ip[1:] - ip[:-1])[sel]
    nip = torch.zeros(sel.numel() + 1, dtype=torch.int64, device=ip.device)
    torch.cumsum(lens, 0, out=nip[1:])
    rid = torch.repeat_interleave(torch.arange(sel.numel(), device=ip.device), lens)
    pos = ip[sel][rid] + torch.arange(rid.numel(), device=ip.device) - nip[rid]
    return nip, ix[pos].contiguous()


def dense_mask_offsets(mask: Tuple[torch.Tensor, torch.Tensor], n_items: int, c0: int, c1: int) -> torch.Tensor:
    """Flat offsets (u - c0) * n_items + item of the masked entries of users [c0, c1) of a mask CSR:
    where score_topk_dense_masked writes -inf into a [c1 - c0, n_items] score block."""
    ip, ix = mask
    sel = torch.arange(c0, c1, device=ip.device)
    sp, sx = csr_rows(mask, sel)
    rid = torch.repeat_interleave(torch.arange(c1 - c0, device=ip.device), sp[1:] - sp[:-1])
    return rid * n_items + sx.to(torch.int64)


# the dense route's f32 score chunk: 1 GiB ranks the long-mask users of the evaluation shapes in one
# chunk (Amazon-book: 737 users, 0.63 -> 0.44 ms against 256 MiB; tools/chunk_probe.py,
# profiles/r05_chunk_probe.txt)
DENSE_CHUNK_BYTES = 1 << 30


def dense_chunk_users(n_items: int, chunk_bytes: int = DENSE_CHUNK_BYTES) -> int:
    return max(1, chunk_bytes // max(1, 4 * n_items))


def score_topk_dense_masked(Q: torch.Tensor, items: torch.Tensor, k: int, user_rows: torch.Tensor,
                            mask: Tuple[torch.Tensor, torch.Tensor], chunk_bytes: int = DENSE_CHUNK_BYTES,
                            offsets: Optional[Sequence[torch.Tensor]] = None,
                            scratch: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The ranking score_topk returns (idx int32 [B, k]; raw scores ranked, ties to the lower item id)
    by another route, for users whose mask is long: their dense raw score rows (lgx_score_dense), the
    masked entries set to -inf, the row top-k (lgx_topk_rows).  In the fused walk every masked item
    of such a user that reaches the running threshold needs an exact test (its 256-bit Bloom filter is
    saturated); here a mask costs one scattered store per item.  Every user must keep at least k
    unmasked items (the fused path's masked tail is not reproduced).  Users go in chunks of at most
    chunk_bytes of scores; offsets: the chunks' dense_mask_offsets, precomputed by a caller that ranks
    the same users again (no host synchronisation then); scratch: a flat f32 buffer of at least
    min(B, chunk users) * n_items elements for the score chunks (a caller on a side stream allocates it
    on its own stream, so the block returns to that stream's pool), else allocated here."""
    require_gpu(Q, items, user_rows)
    B, I = user_rows.numel(), items.shape[0]
    idx = torch.empty((B, k), dtype=torch.int32, device=Q.device)
    step = dense_chunk_users(I, chunk_bytes)
    if scratch is not None and scratch.numel() < min(B, step) * I:
        raise ValueError("score_topk_dense_masked: scratch holds fewer than one chunk of scores")
    for j, c0 in enumerate(range(0, B, step)):
        c1 = min(B, c0 + step)
        S = score_dense(Q, items, user_rows=user_rows[c0:c1],
                        out=scratch[:(c1 - c0) * I].view(c1 - c0, I) if scratch is not None else None)
        off = offsets[j] if offsets is not None else dense_mask_offsets(mask, I, c0, c1)
        S.view(-1).index_fill_(0, off, float("-inf"))
        idx[c0:c1] = topk_rows(S, k)[0]
        del S
    return idx


def score_minmax(Q: torch.Tensor, items: torch.Tensor, user_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Global (min, max) of Q . items^T over every pair (``lgx_score_minmax``) -> f32 [2] on the
    device (recommend.py:163-164, :375-377)."""
    require_gpu(Q, items, user_rows)
    check_pair(Q, items)
    Q = Q.contiguous()
    items = items.contiguous()
    B = user_rows.numel() if user_rows is not None else Q.shape[0]
    if B == 0 or items.shape[0] == 0:
        raise ValueError("score_minmax of an empty matrix")
    rows = user_rows.to(torch.int64).contiguous() if user_rows is not None else None
    dev = Q.device
    L = _lib.lib()
    ws = ctypes.c_size_t(0)
    _lib.check(L.lgx_score_minmax_workspace(B, items.shape[0], ctypes.byref(ws)), "lgx_score_minmax_workspace")
    work = torch.empty(max(ws.value, 1), dtype=torch.uint8, device=dev)
    mm = torch.empty(2, dtype=torch.float32, device=dev)
    _lib.check(L.lgx_score_minmax(Q.data_ptr(), _ptr(rows), items.data_ptr(), B, items.shape[0], Q.shape[1],
                                  _dtype_code(Q), mm.data_ptr(), work.data_ptr(), ws.value, _stream_ptr(dev)),
               "lgx_score_minmax")
    return mm


def topk_rows(S: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row-wise top-k of a dense f32 score matrix (tools.h:13-33); ties -> lower column."""
    require_gpu(S)
    if S.dtype != torch.float32 or S.dim() != 2 or S.stride(1) != 1:
        raise TypeError("topk_rows expects a row-major float32 matrix")
    rows, cols = S.shape
    idx = torch.empty((rows, k), dtype=torch.int32, device=S.device)
    val = torch.empty((rows, k), dtype=torch.float32, device=S.device)
    _lib.check(_lib.lib().lgx_topk_rows(S.data_ptr(), rows, cols, S.stride(0), int(k), idx.data_ptr(), val.data_ptr(),
                                        _stream_ptr(S.device)), "lgx_topk_rows")
    return idx, val


_SMALL_CONST: dict = {}


def _device_const(key: tuple, make) -> torch.Tensor:
    """A small read-only device tensor built once per key (a host-to-device copy per evaluation call
    cost as much as the metric kernel itself)."""
    t = _SMALL_CONST.get(key)
    if t is None:
        t = _SMALL_CONST[key] = make()
    return t


def inv_log2_table(k: int, device) -> torch.Tensor:
    """1.0/log2(i+2) with the host libm (as the C++ evaluator computes it, evaluate_foldout.h:80,84);
    cached per (k, device), read-only."""
    return _device_const(("inv_log2", k, str(torch.device(device))),
                         lambda: torch.tensor([1.0 / math.log2(i + 2) for i in range(k)], dtype=torch.float64,
                                              device=device))


def foldout_metrics(rankings: torch.Tensor, truth: Tuple[torch.Tensor, torch.Tensor]) -> torch.Tensor:
    """evaluate_foldout (evaluate_foldout.h:115-195) -> f32 [users, 5k]."""
    require_gpu(rankings)
    r = rankings.to(torch.int32).contiguous()
    users, k = r.shape
    out = torch.empty((users, 5 * k), dtype=torch.float32, device=r.device)
    tl = inv_log2_table(k, r.device)
    _lib.check(_lib.lib().lgx_foldout_metrics(r.data_ptr(), users, k, truth[0].data_ptr(), truth[1].data_ptr(),
                                              tl.data_ptr(), out.data_ptr(), _stream_ptr(r.device)),
               "lgx_foldout_metrics")
    return out


def column_mean(x: torch.Tensor) -> torch.Tensor:
    """np.mean(x, axis=0) of a float32 [rows, cols] matrix, bit for bit (batch_test.py:75-76): float32
    sums in row order, one float32 division by rows (lgx_column_mean_f32) -> f32 [cols]."""
    require_gpu(x)
    if x.dtype != torch.float32 or x.dim() != 2:
        raise ValueError("column_mean: float32 [rows, cols] expected")
    x = x.contiguous()
    out = torch.empty(x.shape[1], dtype=torch.float32, device=x.device)
    _lib.check(_lib.lib().lgx_column_mean_f32(x.data_ptr(), x.shape[0], x.shape[1], out.data_ptr(),
                                              _stream_ptr(x.device)), "lgx_column_mean_f32")
    return out


def test_metrics(rankings: torch.Tensor, truth: Tuple[torch.Tensor, torch.Tensor], topks: Sequence[int],
                 test_len: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Procedure.Test's metric sums over all users (Procedure.py:60-72, ``lgx_test_metrics``): rankings
    int32 [users, max(topks)], truth = sorted deduplicated test lists as a CSR, test_len = the lists'
    lengths with duplicates (int64 [users]) -> f64 [3, len(topks)] on the device: per topk the sums of
    recall, of right (precision * topk) and of ndcg, in the order of ``topks``.  Any number of topks
    (the reference's list has no limit): the library takes 8 per launch, so longer lists go in groups."""
    require_gpu(rankings)
    r = rankings.to(torch.int32).contiguous()
    users, k = r.shape
    ks = [int(x) for x in topks]
    if not ks or min(ks) < 1 or max(ks) != k:
        raise ValueError(f"test_metrics: topks {ks} with rankings of width {k} (each in 1..width, max = width)")
    if len(ks) > 8:
        parts = [_test_metrics_group(r, truth, ks[g:g + 8], test_len) for g in range(0, len(ks), 8)]
        return torch.cat(parts, dim=1)
    return _test_metrics_group(r, truth, ks, test_len)


def _test_metrics_group(r: torch.Tensor, truth, ks, test_len) -> torch.Tensor:
    """test_metrics for at most 8 topks, each in [1, width] (the lgx_test_metrics contract)."""
    users, k = r.shape
    order = sorted(range(len(ks)), key=lambda i: ks[i])
    tk = _device_const(("topks", tuple(ks[i] for i in order), str(r.device)),
                       lambda: torch.tensor([ks[i] for i in order], dtype=torch.int32, device=r.device))
    tl = inv_log2_table(k, r.device)
    L = _lib.lib()
    ws = ctypes.c_size_t(0)
    _lib.check(L.lgx_test_metrics_workspace(users, len(ks), ctypes.byref(ws)), "lgx_test_metrics_workspace")
    work = torch.empty(max(ws.value, 8), dtype=torch.uint8, device=r.device)
    out = torch.empty((len(ks), 3), dtype=torch.float64, device=r.device)
    tlen = test_len.to(torch.int64).contiguous() if test_len is not None else None
    _lib.check(L.lgx_test_metrics(r.data_ptr(), users, k, truth[0].data_ptr(), truth[1].data_ptr(), _ptr(tlen),
                                  tk.data_ptr(), len(ks), tl.data_ptr(), out.data_ptr(), work.data_ptr(), ws.value,
                                  _stream_ptr(r.device)), "lgx_test_metrics")
    if order == list(range(len(ks))):
        return out.t()
    inv = _device_const(("topks_inv", tuple(order), str(r.device)),
                        lambda: torch.tensor(order, device=r.device).argsort())
    return out[inv].t()


def gather_scores(emb_user: torch.Tensor, emb_item: torch.Tensor, cand: Tuple[torch.Tensor, torch.Tensor],
                  n_pairs: int) -> torch.Tensor:
    """Per-user candidate dots (recommend.py:167-171, :214-217) -> f32 [n_pairs].  List u is scored
    against emb_user row u, so there must be at most emb_user.shape[0] lists; a candidate id outside
    the item table raises IndexError, as the reference's numpy indexing does."""
    require_gpu(emb_user, emb_item)
    eu = emb_user.to(torch.float32).contiguous()
    ei = emb_item.to(torch.float32).contiguous()
    n_lists = int(cand[0].numel()) - 1
    if n_lists < 0 or n_lists > eu.shape[0]:
        raise ValueError(f"{n_lists} candidate lists for {eu.shape[0]} user rows")
    if n_pairs and cand[1].numel():
        items = cand[1][:n_pairs]
        lo, hi = int(items.min()), int(items.max())
        if lo < 0 or hi >= ei.shape[0]:
            raise IndexError(f"candidate item id {lo if lo < 0 else hi} out of range for {ei.shape[0]} items")
    out = torch.empty(max(n_pairs, 1), dtype=torch.float32, device=eu.device)
    _lib.check(_lib.lib().lgx_gather_scores(eu.data_ptr(), ei.data_ptr(), n_lists, ei.shape[0], eu.shape[1],
                                            cand[0].data_ptr(), cand[1].data_ptr(), n_pairs, out.data_ptr(),
                                            _stream_ptr(eu.device)),
               "lgx_gather_scores")
    return out[:n_pairs]


def fill_normal(shape, std: float, seed: int, dtype=torch.float32, device="cuda", first: int = 0) -> torch.Tensor:
    """Deterministic N(0, std^2) table; `first` = flat offset into the seeded sequence, so
    fill_normal((r1 - r0, d), ..., first=r0 * d) equals rows [r0, r1) of the full table."""
    t = torch.empty(shape, dtype=dtype, device=device)
    require_gpu(t)
    L, sd = _lib.lib(), int(seed) & (2**64 - 1)
    rc = (L.lgx_fill_normal(t.data_ptr(), t.numel(), float(std), sd, _dtype_code(t), _stream_ptr(t.device))
          if first == 0 else
          L.lgx_fill_normal_at(t.data_ptr(), int(first), t.numel(), float(std), sd, _dtype_code(t),
                               _stream_ptr(t.device)))
    _lib.check(rc, "lgx_fill_normal")
    return t


# ------------------------------------------------------------------------------------ BPR loss
def _bpr_args(light, ego_user, ego_item, users, pos, neg):
    require_gpu(light, ego_user, ego_item, users, pos, neg)
    for t in (light, ego_user, ego_item):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("light / ego tables must be contiguous float32")
    U, I = ego_user.shape[0], ego_item.shape[0]
    d = light.shape[1]
    if light.shape[0] != U + I or ego_user.shape[1] != d or ego_item.shape[1] != d:
        raise ValueError(f"shape mismatch: light {tuple(light.shape)}, ego {tuple(ego_user.shape)} / "
                         f"{tuple(ego_item.shape)}")
    idx = [t.contiguous().long() for t in (users, pos, neg)]
    if not (idx[0].shape == idx[1].shape == idx[2].shape) or idx[0].dim() != 1 or idx[0].numel() == 0:
        raise ValueError("users / pos / neg must be equal-length non-empty 1-D index tensors")
    return U, I, d, idx


def bpr_loss_forward(light: torch.Tensor, ego_user: torch.Tensor, ego_item: torch.Tensor, users: torch.Tensor,
                     pos: torch.Tensor, neg: torch.Tensor):
    """``lgx_bpr_loss_forward`` (model.py:196-209): returns (loss, reg_loss, coef) -- two 0-dim f32
    tensors and the per-triple sigmoid(<u,n> - <u,p>) the backward needs.  light = the propagated
    [U+I, d] table, ego_* = the embedding weights."""
    U, I, d, (u, p, n) = _bpr_args(light, ego_user, ego_item, users, pos, neg)
    B = u.numel()
    sz = ctypes.c_size_t()
    _lib.check(_lib.lib().lgx_bpr_loss_workspace(B, ctypes.byref(sz)), "lgx_bpr_loss_workspace")
    ws = torch.empty(sz.value, dtype=torch.uint8, device=light.device)
    coef = torch.empty(B, dtype=torch.float32, device=light.device)
    loss = torch.empty((), dtype=torch.float32, device=light.device)
    reg = torch.empty((), dtype=torch.float32, device=light.device)
    _lib.check(_lib.lib().lgx_bpr_loss_forward(light.data_ptr(), ego_user.data_ptr(), ego_item.data_ptr(), U, I, d,
                                               u.data_ptr(), p.data_ptr(), n.data_ptr(), B, coef.data_ptr(),
                                               loss.data_ptr(), reg.data_ptr(), ws.data_ptr(), sz.value,
                                               _stream_ptr(light.device)), "lgx_bpr_loss_forward")
    return loss, reg, coef


def bpr_loss_backward(light, ego_user, ego_item, users, pos, neg, coef, grad_loss, grad_reg):
    """``lgx_bpr_loss_backward``: dense gradients (g_light [U+I, d], g_user [U, d], g_item [I, d]) of
    grad_loss * loss + grad_reg * reg (0-dim device tensors)."""
    U, I, d, (u, p, n) = _bpr_args(light, ego_user, ego_item, users, pos, neg)
    g_light = torch.zeros_like(light)
    g_user = torch.zeros_like(ego_user)
    g_item = torch.zeros_like(ego_item)
    gl = grad_loss.to(torch.float32).contiguous()
    gr = grad_reg.to(torch.float32).contiguous()
    _lib.check(_lib.lib().lgx_bpr_loss_backward(light.data_ptr(), ego_user.data_ptr(), ego_item.data_ptr(), U, I, d,
                                                u.data_ptr(), p.data_ptr(), n.data_ptr(), u.numel(), coef.data_ptr(),
                                                gl.data_ptr(), gr.data_ptr(), g_light.data_ptr(), g_user.data_ptr(),
                                                g_item.data_ptr(), _stream_ptr(light.device)), "lgx_bpr_loss_backward")
    return g_light, g_user, g_item


# ------------------------------------------------------------------------------------ introspection
def spmm_kernel_name(d: int, dtype: torch.dtype, seg_len: int) -> str:
    """The SpMM instantiation lgx_propagate_layer launches for this embedding dim / storage dtype /
    plan segment length (``lgx_spmm_kernel_name``; host only)."""
    buf = ctypes.create_string_buffer(256)
    code = _lib.LGX_DTYPE_BF16 if dtype == torch.bfloat16 else _lib.LGX_DTYPE_F32
    _lib.check(_lib.lib().lgx_spmm_kernel_name(int(d), code, int(seg_len), buf, 256), "lgx_spmm_kernel_name")
    return buf.value.decode()


def score_topk_plan(B: int, n_items: int, d: int, dtype: torch.dtype, k: int) -> str:
    """The launch plan of lgx_score_topk for this shape (``lgx_score_topk_plan``; host only)."""
    buf = ctypes.create_string_buffer(1024)
    code = _lib.LGX_DTYPE_BF16 if dtype == torch.bfloat16 else _lib.LGX_DTYPE_F32
    _lib.check(_lib.lib().lgx_score_topk_plan(int(B), int(n_items), int(d), code, int(k), buf, 1024),
               "lgx_score_topk_plan")
    return buf.value.decode()
