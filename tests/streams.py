"""Adversarial string-record streams for the index-free decode (pure numpy:
used by tests/test_gpu_stream.py and tools/stream_bench.py)."""
import numpy as np


def straddler_stream(n, rng, lead, over, fill="zero", maxlen=24, p_empty=0.5, p_nonzero=0.05):
    """zero-heavy int8/string/int16/string records,
    and across EVERY 8 KiB block boundary one record (its first string
    `fill`: all zero bytes, or zero-heavy like the rest) that starts `lead`
    bytes before the boundary and ends `over` bytes after it -- past the
    table's 64-byte window, inside chars where the speculation has no clue.
    Returns the columns and string offsets for oracle.pack."""
    l0 = rng.integers(0, maxlen, n)
    l0[rng.random(n) < p_empty] = 0
    l1 = rng.integers(0, maxlen, n)
    l1[rng.random(n) < p_empty] = 0
    size = 19 + l0 + l1
    pos, i, B = 0, 0, 8192
    L0, L1, FIL = [], [], []
    while i < n:
        ld, ov = int(rng.integers(*lead)), int(rng.integers(*over))
        cs = pos + np.cumsum(size[i:i + 2 * 8192 // 19 + 4])
        k = min(int(np.searchsorted(cs, B - ld, side="right")), n - i)
        L0.append(l0[i:i + k])
        L1.append(l1[i:i + k])
        FIL.append(np.zeros(k, bool))
        if k:
            pos = int(cs[k - 1])
        i += k
        if i >= n:
            break
        L0.append(np.array([B + ov - pos - 19]))  # from pos (at most `lead` before B) to B + over
        L1.append(np.array([0]))
        FIL.append(np.ones(1, bool))
        pos, i = B + ov, i + 1
        while B <= pos:
            B += 8192
    l0, l1, fil = np.concatenate(L0)[:n], np.concatenate(L1)[:n], np.concatenate(FIL)[:n]
    cols, offs = [np.zeros(n, np.int8), None, np.zeros(n, np.int16), None], [None, None, None, None]
    for f, ls in ((1, l0), (3, l1)):
        o = np.zeros(n + 1, np.uint64)
        o[1:] = np.cumsum(ls)
        c = np.zeros(max(1, int(o[-1])), np.uint8)
        nz = rng.random(c.size) < p_nonzero
        if fill == "zero":  # the straddling records' chars stay all zero
            for r in np.flatnonzero(fil & (ls > 0)):
                nz[int(o[r]):int(o[r + 1])] = False
        c[nz] = 7
        cols[f], offs[f] = c, o
    return cols, offs
