"""GPU: interaction-file parsing (dataloader.py:247-277 / load_data.py:27-48) against a Python
tokenizer of the same grammar, on the mlls files, on edge cases, and on a multi-chunk file with
numbers and lines that straddle the 64-KiB chunk boundaries."""
import numpy as np
import pytest
import torch

from factors_of_serendipity_recommendation_amd import ops
from factors_of_serendipity_recommendation_amd.dataloader import read_interactions

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _py_parse(text: bytes):
    users, ptr, items = [], [0], []
    for line in text.split(b"\n"):
        nums, cur = [], None
        for c in line:
            if 48 <= c <= 57:
                cur = (cur or 0) * 10 + (c - 48)
            elif cur is not None:
                nums.append(cur)
                cur = None
        if cur is not None:
            nums.append(cur)
        if nums:
            users.append(nums[0])
            items.extend(nums[1:])
            ptr.append(len(items))
    return users, ptr, items


def _check(text: bytes):
    lu, lp, it, pu = ops.parse_lines(torch.from_numpy(np.frombuffer(text, dtype=np.uint8).copy()).to(DEV))
    users, ptr, items = _py_parse(text)
    assert lu.cpu().tolist() == users
    assert lp.cpu().tolist() == ptr
    assert it.cpu().tolist() == items
    assert pu.cpu().tolist() == [u for u, a, b in zip(users, ptr[:-1], ptr[1:]) for _ in range(b - a)]


def test_parse_edge_cases():
    _check(b"")
    _check(b"\n\n")
    _check(b"7")
    _check(b"0 1 2 3\n4 5\n")
    _check(b"0 1 2 3\r\n4 5\r\n6\r\n\r\n  8   9 10  \n11 12")  # CRLF, blank, leading/trailing blanks, no final \\n
    _check(b"3\n4 99999\n")  # a line with only its user


def test_parse_multichunk_random():
    rng = np.random.default_rng(0)
    lines = []
    for u in range(30000):
        k = int(rng.integers(0, 30))
        lines.append(" ".join(str(x) for x in [u] + rng.integers(0, 10 ** int(rng.integers(1, 9)), k).tolist()))
    text = ("\n".join(lines) + "\n").encode()
    assert len(text) > 10 * 65536
    _check(text)


def test_loader_files_match_oracle_parser(mlls, tmp_path):
    """The GPU reader against the oracle's restatement of Loader.__init__ (dataloader.py:247-285)."""
    from oracle import oracle
    tp, tx = mlls["train_list_indptr"], mlls["train_list_indices"]
    path = tmp_path / "train.txt"
    with open(path, "w") as f:
        for j, u in enumerate(mlls["train_list_users"]):
            f.write(" ".join(str(x) for x in [u] + list(tx[tp[j]:tp[j + 1]])) + "\n")
    sp_, sx = mlls["test_indptr"], mlls["test_indices"]
    tpath = tmp_path / "test.txt"
    with open(tpath, "w") as f:
        for j, u in enumerate(mlls["test_users"]):
            f.write(" ".join(str(x) for x in [u] + list(sx[sp_[j]:sp_[j + 1]])) + "\n")
    ou, oi, otest, on_u, on_i, otrain = oracle.parse_lightgcn_txt(str(path), str(tpath))
    gu, gr = read_interactions(str(path), DEV)
    assert gu == list(otrain.keys())
    assert all(np.array_equal(r, otrain[u]) for u, r in zip(gu, gr))
    assert np.array_equal(np.concatenate(gr), np.asarray(oi))
