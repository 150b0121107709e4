"""The C++ API mirror (include/srpc/*.hpp): the reference's packer/server tests
restated against our headers, the reference's generated example compiled
unchanged against them (build container only), and -- on a GPU -- the
srpc::gpu::batch_packer<T> batch API against the scalar packer."""
import os
import subprocess

import pytest

from tests.cpp import build_cpp

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(name, timeout=120):
    src = os.path.join(HERE, "cpp", name + ".cpp")
    exe = build_cpp.build_one(src)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stdout + out.stderr
    return out.stdout


def test_cpp_packer_and_server():
    assert "0 failed" in _run("packer_test")


@pytest.mark.skipif(not os.path.isdir(os.path.join(build_cpp.REF, "examples")),
                    reason="reference tree absent (GPU box)")
def test_reference_generated_stub_links_unchanged():
    assert "ok" in _run("calculator_compat_test")


def test_cpp_schema_limits_refused():
    """33 leaf fields or a 1025-byte envelope: batch_packer<T> throws plan_error
    with SRPC_E_UNSUPPORTED (refused before any device work, so no GPU needed)."""
    from srpc_amd import build
    build.build()
    out = _run("schema_limits_test")
    assert "0 failed" in out and out.count("refused:") == 3


def test_cpp_multi_gpu_api_compiles():
    """sharded_packer<T>::request, pack_gather, comm / device_group moves:
    instantiated and linked against libsrpc_gpu.so, not called (no GPU)."""
    from srpc_amd import build
    build.build()
    assert "ok" in _run("multi_api_compile_test")


@pytest.mark.gpu
def test_cpp_gpu_batch_packer():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from srpc_amd import build
    build.build()
    assert "0 failed" in _run("gpu_batch_test", timeout=300)
