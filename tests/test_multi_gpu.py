"""Native multi-GPU path of the library (include/srpc_gpu.h srpc_comm_*,
srpc_gather_wire, srpc_group_pack_gather; include/srpc/gpu_multi.hpp): on
every visible MI355X a sharded pack gathered to device 0 over RCCL equals the
single-device pack.  The box has one GPU: the group machinery runs end to end
with the root's own shard; the 8-GPU exchange is measured by bench.py."""
import os
import subprocess

import pytest

from tests.cpp import build_cpp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_sharded_packer_cpp():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    src = os.path.join(HERE, "cpp", "multi_gpu_test.cpp")
    exe = build_cpp.exe_path(src)
    if not os.path.exists(exe):
        exe = build_cpp.build_one(src)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "0 failed" in out.stdout, out.stdout + out.stderr


def test_native_comm_python_one_rank():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from srpc_amd.shard import NativeComm
    c = NativeComm(NativeComm.unique_id(), 1, 0, 0)
    local = torch.arange(1000, dtype=torch.int32, device="cuda:0").view(torch.uint8)
    out = c.gather_wire(local, [local.numel()], 0)
    torch.cuda.synchronize()
    assert torch.equal(out, local)
    c.close()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("n", [17, 4099, 100_003])
def test_shards_concatenate_to_the_batch(world, n):
    """The reference appends records to one buffer (core.hpp:34, packer.hpp:73),
    so the wire of a batch is the concatenation of its shards' wires: every
    rank's srpc_shard_range slice (16-record aligned cuts) packed on its own --
    here all on device 0 -- and laid end to end equals the oracle's batch,
    for fixed records (Quad) and for string records (offsets sliced, chars
    shared: each shard's offsets start wherever its first record's chars do)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import numpy as np

    import oracle
    from srpc_amd import QUAD, GpuPacker, Schema
    from srpc_amd.shard import native_shard_range
    from tests.test_gpu_parity import _dev_u64, _random_string_batch, dev, empty, host

    cols = oracle.splitmix_columns_i32(4, n)
    p = GpuPacker(QUAD)
    dcols = [dev(c) for c in cols]
    parts = []
    for r in range(world):
        lo, hi = native_shard_range(n, r, world)
        assert lo % 16 == 0 and (hi % 16 == 0 or hi == n)
        w = empty(16 * (hi - lo) + 16)
        if hi > lo:
            p.pack([c[4 * lo:4 * hi] for c in dcols], hi - lo, w)
        parts.append(host(w, 16 * (hi - lo)).tobytes())
    assert b"".join(parts) == oracle.pack([oracle.INT32] * 4, cols, n)

    kinds = [oracle.INT8, oracle.STRING, oracle.INT64]
    scols, soffs = _random_string_batch(kinds, n, np.random.default_rng(n + world), 40)
    sp = GpuPacker(Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds))))
    want = oracle.pack(kinds, scols, n, b"", list(soffs))
    dc = [dev(scols[0]), dev(scols[1]), dev(scols[2])]
    doff = _dev_u64(soffs[1])
    parts = []
    for r in range(world):
        lo, hi = native_shard_range(n, r, world)
        m = hi - lo
        total = 17 * m + int(soffs[1][hi] - soffs[1][lo])
        w, rec = empty(total + 16), empty(8 * (m + 1))
        sb = sp.var_scratch_bytes(m, total)
        scratch = empty(sb + 16)
        if m:
            sp.pack_var([dc[0][lo:hi], dc[1], dc[2][8 * lo:8 * hi]], [None, doff[8 * lo:8 * (hi + 1)], None], m, w,
                        total, rec, scratch, sb)
        parts.append(host(w, total).tobytes())
    assert b"".join(parts) == want
