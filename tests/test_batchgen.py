"""srpc_amd.batchgen: contract parsing, the emitted batch
views and message structs (golden header), their use by the scalar packer
(host C++), and -- on a GPU -- by the batch path."""
import hashlib
import os
import subprocess

import pytest

from srpc_amd import batchgen
from tests.cpp import build_cpp

HERE = os.path.dirname(os.path.abspath(__file__))
CONTRACT = os.path.join(HERE, "cpp", "batchgen_example.contract")
REF_CONTRACT = os.path.join(build_cpp.REF, "examples", "calculator.contract")


def _contract():
    return batchgen.parse(open(CONTRACT).read())


def test_parse_and_flatten():
    c = _contract()
    assert [m.name for m in c.messages] == ["Inner", "Point", "Number", "Record"]
    rec = c.message("Record")
    assert batchgen.flatten(c, rec) == [("id", "int64"), ("in_tag", "int8"), ("in_small", "int16"),
                                        ("flag", "bool"), ("label", "string"), ("c", "char"),
                                        ("p_x", "int32"), ("p_y", "int32"), ("note", "string")]
    (svc,) = c.services
    assert [(m.name, m.input_t, m.output_t) for m in svc.methods] == [("locate", "Point", "Record"),
                                                                       ("square", "Number", "Number")]


@pytest.mark.parametrize("text,err", [
    ("message A { int32 x }", "expected ';'"),
    ("message A { Foo x; }", "Undefined identifier"),
    ("message A { A x; }", "Undefined identifier"),
    ("message A { int32 name; }", "collides"),
    ("message A { int32 x; int8 x; }", "repeated"),
    ("message A { int32 x; } message A { int8 y; }", "defined twice"),
    ("service S { method m(Nope) returns (Nope); }", "Undefined message type"),
    ("msg A { }", "expected 'message' or 'service'"),
    ("message A { int32 message; }", "identifier"),
])
def test_parse_errors(text, err):
    with pytest.raises(batchgen.ContractError, match=err):
        batchgen.parse(text)


def test_generated_header_matches_golden():
    want = open(os.path.join(HERE, "golden", "batchgen_example_batch.hpp")).read()
    assert batchgen.generate(_contract(), "batchgen_example.contract", messages=True) == want


def test_cli_writes_header(tmp_path):
    out = tmp_path / "x_batch.hpp"
    assert batchgen.main([CONTRACT, "-o", str(out)]) == 0
    text = out.read_text()
    assert "struct Record_batch" in text and "struct Record :" not in text  # companions only
    bad = tmp_path / "bad.contract"
    bad.write_text("message A { Foo x; }")
    assert batchgen.main([str(bad), "-o", str(tmp_path / "b.hpp")]) == 1


def test_generated_messages_with_scalar_packer():
    exe = build_cpp.build_one(os.path.join(HERE, "cpp", "batchgen_host_test.cpp"))
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "0 failed" in out.stdout, out.stdout + out.stderr


@pytest.mark.skipif(not os.path.exists(REF_CONTRACT), reason="reference tree absent (GPU box)")
def test_companions_compile_with_reference_generated_stubs(tmp_path):
    """calculator.contract -> calculator_batch.hpp, included after the
    reference's generated calculator_srpc.cpp, compiles against our headers."""
    hdr = tmp_path / "calculator_batch.hpp"
    assert batchgen.main([REF_CONTRACT, "-o", str(hdr)]) == 0
    src = tmp_path / "use.cpp"
    src.write_text('#include "calculator_srpc.cpp"\n#include "calculator_batch.hpp"\n'
                   "int main() { Number_batch b; auto p = Calculator_batch::square_request; (void)p;\n"
                   "  return static_cast<int>(b.nfields + TwoNumbers_batch::nfields) - 3; }\n")
    cmd = ["g++", "-std=c++20", "-fsyntax-only", "-I", os.path.join(build_cpp.ROOT, "include"),
           "-I", os.path.join(build_cpp.REF, "examples"), "-I", str(tmp_path), str(src)]
    out = subprocess.run(cmd, capture_output=True, text=True)
    assert out.returncode == 0, out.stderr


@pytest.mark.gpu
def test_generated_batch_views_on_gpu(tmp_path, manifest):
    """The generated Record_batch / Point_batch views packed on the GPU give
    exactly the bytes the REFERENCE packer produced for the same records
    (tests/cpp/geo_records.hpp; digests from oracle/ref_shim.cpp via
    tests/golden/make_golden.py), and unpack gives the columns back."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = build_cpp.exe_path(os.path.join(HERE, "cpp", "batchgen_gpu_test.cpp"))
    if not os.path.exists(exe):  # built in the build container (build_cpp.build_all)
        exe = build_cpp.build_one(os.path.join(HERE, "cpp", "batchgen_gpu_test.cpp"))
    out = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "0 failed" in out.stdout, out.stdout + out.stderr
    ref = manifest["batchgen"]
    for label in ("geo_locate_responses", "geo_locate_requests"):
        got = (tmp_path / f"{label}.bin").read_bytes()
        assert len(got) == ref[label]["bytes"], label
        assert hashlib.sha256(got).hexdigest() == ref[label]["sha256"], label
