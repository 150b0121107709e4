"""The library inside a hipGraph stream capture.

Round 4 captured bench.py's whole PCIe pipeline with torch.cuda.graph and the
process died in the capture; tools/capture_probe.py took that capture apart
(profiles/r05_capture_probe.json).  What the library itself
promises is tested here: its device calls (DWORD and TILE packs and unpacks,
an enveloped layout, the host-terminated direct mode on mapped pinned memory)
are captured and replayed with the same bytes as eager calls, and the chunked
host-terminated mode -- which would pull the library's own streams into the
caller's graph -- refuses a capturing stream with SRPC_E_UNSUPPORTED before it
enqueues anything, so the capture still ends cleanly."""
import numpy as np
import pytest

import oracle
import srpc_amd
from srpc_amd import QUAD, GpuPacker, Schema

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("no GPU", allow_module_level=True)

ALL = [oracle.BOOL, oracle.INT8, oracle.CHAR, oracle.INT16, oracle.INT32, oracle.INT64]
NP = {oracle.BOOL: np.uint8, oracle.INT8: np.int8, oracle.CHAR: np.uint8, oracle.INT16: np.int16,
      oracle.INT32: np.int32, oracle.INT64: np.int64}


def _cols(kinds, n, rng):
    out = []
    for k in kinds:
        a = rng.integers(0, 256, n * oracle.KIND_SIZE[k], dtype=np.uint8).view(NP[k]).copy()
        if k == oracle.BOOL:
            a &= 1
        out.append(a)
    return out


@pytest.mark.parametrize("which", ["quad", "all_request"])
def test_device_calls_captured_and_replayed(which):
    if which == "quad":
        kinds, p = QUAD.kinds, GpuPacker(QUAD)
    else:
        kinds = ALL
        p = GpuPacker.for_request(Schema("S", tuple((f"f{i}", k) for i, k in enumerate(ALL))), "Svc_servicer::m")
    n = 100_003
    host_cols = _cols(kinds, n, np.random.default_rng(11))
    want = bytes(oracle.pack(kinds, host_cols, n, p.prefix))
    cols = [torch.from_numpy(c.view(np.uint8)).cuda() for c in host_cols]
    back = [torch.zeros_like(c) for c in cols]
    wire = torch.zeros(len(want) + 16, dtype=torch.uint8, device="cuda")
    st = torch.zeros(16, dtype=torch.uint8, device="cuda")
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=side):
        cur = torch.cuda.current_stream()
        p.pack(cols, n, wire, stream=cur)
        p.unpack(wire, len(want), n, back, status=st, stream=cur)
    torch.cuda.synchronize()
    assert not wire[:len(want)].any()  # capturing ran nothing
    g.replay()
    torch.cuda.synchronize()
    assert wire[:len(want)].cpu().numpy().tobytes() == want
    for a, b in zip(cols, back):
        assert torch.equal(a, b)
    assert st[:4].cpu().numpy().view(np.uint32)[0] == 0
    # a second replay after the inputs change: the graph reads them again
    cols[0].zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(back[0], cols[0])


def test_host_direct_captured_chunked_refused():
    p = GpuPacker(QUAD)
    n = 65_536
    host_cols = _cols(QUAD.kinds, n, np.random.default_rng(12))
    want = bytes(oracle.pack(QUAD.kinds, host_cols, n))
    h_cols = [torch.from_numpy(c.view(np.uint8)).pin_memory() for c in host_cols]
    h_wire = torch.zeros(len(want), dtype=torch.uint8).pin_memory()
    sb = p.host_scratch_bytes(n // 4, 2)
    scr = torch.empty(sb + 256, dtype=torch.uint8, device="cuda")
    sp = scr.data_ptr() + (-scr.data_ptr()) % 256
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    refused = None
    with torch.cuda.graph(g, stream=side):
        cur = torch.cuda.current_stream()
        p.pack_host([h.data_ptr() for h in h_cols], n, h_wire, 0, 0, 0, depth=1, stream=cur)  # direct: captured
        try:
            p.pack_host([h.data_ptr() for h in h_cols], n, h_wire, n // 4, sp, sb, depth=2, stream=cur)
        except srpc_amd.SrpcError as e:
            refused = e
    assert refused is not None and "not supported" in str(refused)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert h_wire.numpy().tobytes() == want


def test_stream_decode_captured_and_replayed():
    """The index-free stream decode (five launches, scratch in the caller's
    buffer, nothing read back to the host) captured once and replayed:
    columns and offsets equal the oracle's, and again after the outputs are
    cleared."""
    from tests.test_gpu_parity import _random_string_batch
    kinds = [oracle.INT8, oracle.STRING, oracle.INT16, oracle.STRING]
    p = GpuPacker(Schema("zh4", tuple((f"f{i}", k) for i, k in enumerate(kinds))))
    n = 200_003
    rng = np.random.default_rng(21)
    cols, offs = _random_string_batch(kinds, n, rng, 24)
    wire = bytes(oracle.pack(kinds, cols, n, b"", offs))
    W = len(wire)
    rc, ocols, ooffs, _, _ = oracle.unpack(kinds, wire, n, b"")
    assert rc == oracle.ORC_OK
    d_wire = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).cuda()
    outs = [torch.zeros(W + 16 if k == oracle.STRING else n * oracle.KIND_SIZE[k] + 16, dtype=torch.uint8,
                        device="cuda") for k in kinds]
    soffs = [torch.zeros(8 * (n + 1), dtype=torch.uint8, device="cuda") if k == oracle.STRING else None
             for k in kinds]
    rec = torch.zeros(8 * (n + 1), dtype=torch.uint8, device="cuda")
    sb = p.var_stream_scratch_bytes(n, W)
    scr = torch.empty(sb + 256, dtype=torch.uint8, device="cuda")
    sp = scr.data_ptr() + (-scr.data_ptr()) % 256
    st = torch.zeros(16, dtype=torch.uint8, device="cuda")
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=side):
        p.unpack_var_stream(d_wire, W, n, rec, outs, soffs, sp, sb, st, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert not rec.any()  # capturing ran nothing

    def check(ocols, ooffs):
        for f, k in enumerate(kinds):
            if k == oracle.STRING:
                oh = soffs[f].cpu().numpy().view(np.uint64)
                assert np.array_equal(oh, ooffs[f]), f
                assert outs[f][:int(oh[n])].cpu().numpy().tobytes() == ocols[f].tobytes(), f
            else:
                got = outs[f][:n * oracle.KIND_SIZE[k]].cpu().numpy().tobytes()
                assert got == ocols[f].tobytes(), f
        assert st[:4].cpu().numpy().view(np.uint32)[0] == 0

    g.replay()
    torch.cuda.synchronize()
    check(ocols, ooffs)
    # outputs cleared, replayed again: the graph writes them again
    for o in outs:
        o.zero_()
    rec.zero_()
    g.replay()
    torch.cuda.synchronize()
    check(ocols, ooffs)
