"""Vectorised writer of LightGCN ``uid item item ...`` text (test helper): numbers are turned into
ASCII digits column by column with numpy, so a 10^7-10^8 pair file is written in seconds."""
import numpy as np


def lines_to_bytes(uids: np.ndarray, offsets: np.ndarray, items: np.ndarray) -> bytes:
    """One line per uid: ``uid item item ...\\n`` (items[offsets[j]:offsets[j+1]])."""
    uids = np.asarray(uids, dtype=np.int64)
    offsets = np.asarray(offsets, dtype=np.int64)
    items = np.asarray(items, dtype=np.int64)
    L = len(uids)
    lens = np.diff(offsets)
    # number stream: uid_j followed by its items
    start_of_line = offsets[:-1] + np.arange(L)          # index of uid_j in the number stream
    nums = np.empty(L + len(items), dtype=np.int64)
    is_uid = np.zeros(len(nums), dtype=bool)
    is_uid[start_of_line] = True
    nums[is_uid] = uids
    nums[~is_uid] = items
    last = np.zeros(len(nums), dtype=bool)
    last[start_of_line + lens] = True                     # last number of each line
    nd = np.ones(len(nums), dtype=np.int64)
    p = np.int64(10)
    while True:
        more = nums >= p
        if not more.any():
            break
        nd += more
        p *= 10
    width = nd + 1                                        # digits + separator
    pos = np.zeros(len(nums) + 1, dtype=np.int64)
    np.cumsum(width, out=pos[1:])
    buf = np.empty(int(pos[-1]), dtype=np.uint8)
    rem = nums.copy()
    for k in range(int(nd.max())):                        # k-th digit from the right
        m = nd > k
        buf[pos[:-1][m] + nd[m] - 1 - k] = (rem[m] % 10 + 48).astype(np.uint8)
        rem //= 10
    buf[pos[1:] - 1] = np.where(last, 10, 32).astype(np.uint8)
    return buf.tobytes()
