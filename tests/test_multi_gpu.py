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
