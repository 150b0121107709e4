"""The adversarial straddler streams (tests/streams.py) are what DESIGN §4.4.1
says they are: across every 8 KiB block edge one record that starts within
`lead` bytes before the edge and ends `over` bytes past it (past the decode
table's 64-byte window), its chars zero-filled or zero-heavy.  CPU only: the
records are located with the oracle's own unpack (the reference cursor)."""
import numpy as np
import pytest

import oracle
from tests.streams import straddler_stream

KINDS = [oracle.INT8, oracle.STRING, oracle.INT16, oracle.STRING]


@pytest.mark.parametrize("lead,over,fill", [((1, 960), (65, 1000), "zero"), ((1, 900), (65, 100), "heavy"),
                                            ((1, 6000), (65, 6000), "zero")])
def test_every_block_edge_is_straddled(lead, over, fill):
    n = 30_000
    cols, offs = straddler_stream(n, np.random.default_rng(5), lead, over, fill)
    wire = bytes(oracle.pack(KINDS, cols, n, b"", offs))
    rc, ocols, ooffs, consumed, _ = oracle.unpack(KINDS, wire, n, b"")
    assert rc == oracle.ORC_OK and consumed == len(wire)
    # record starts from the field sizes: 1 + 8 + len0 + 2 + 8 + len1
    l0 = np.diff(ooffs[1].astype(np.int64))
    l1 = np.diff(ooffs[3].astype(np.int64))
    ends = np.cumsum(19 + l0 + l1)
    starts = ends - (19 + l0 + l1)
    assert ends[-1] == len(wire)
    B = 8192
    seen = 0
    while B < ends[-1] - 8192:
        r = int(np.searchsorted(ends, B, side="right"))  # the record that holds byte B
        if starts[r] == B:  # a record starting exactly at the edge is no straddler
            B += 8192
            continue
        # (the last ordinary record ends at most `lead` before the edge, so
        # the straddler starts up to one ordinary record, <= 65 bytes, earlier)
        assert B - starts[r] <= lead[1] + 65, (B, starts[r])
        # it ends past the table window (or, for the long leads, the record
        # spans more than one edge: the next edge is inside it)
        assert ends[r] - B >= over[0] or ends[r] > B + 8192, (B, ends[r])
        if fill == "zero":
            s0 = int(ooffs[1][r])
            assert not ocols[1][s0:s0 + int(l0[r])].any()  # zero-filled chars
        seen += 1
        B += 8192
    assert seen >= (ends[-1] // 8192) // 2
