"""Host AddressSanitizer / UndefinedBehaviorSanitizer builds.

The reference reads before it checks (packer.hpp:212-213 vs core.hpp:29-31);
the CPU restatement (oracle/packer_oracle.c) and this repository's scalar C++
packer (include/srpc/*.hpp) claim to check first.  Both are built here with
-fsanitize=address,undefined (host code only; GPU sanitizers are not
available) and driven through truncated streams cut at every length,
oversized string lengths, foreign prefixes and short output buffers:
tests/cpp/oracle_sanitize_test.c and tests/cpp/packer_test.cpp (the
reference's packer/server tests restated, plus a truncation sweep).  Where
the reference tree exists, its generated calculator stubs compiled against
our headers run end to end under the sanitizers too.
"""
import os
import subprocess

import pytest

from tests.cpp import build_cpp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _run(exe, *args, ok="0 failed"):
    out = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=ENV)
    assert out.returncode == 0 and ok in out.stdout, out.stdout + out.stderr
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr


def _build(tmp_path, cmd):
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0 and "asan" in (out.stderr.lower()) and "cannot find" in out.stderr.lower():
        pytest.skip("sanitizer runtime not installed")
    assert out.returncode == 0, out.stderr


def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_san")
    _build(tmp_path, ["gcc", "-std=c11", *SAN, "-o", exe, os.path.join(HERE, "cpp", "oracle_sanitize_test.c"),
                      os.path.join(ROOT, "oracle", "packer_oracle.c")])
    _run(exe)


def test_cpp_packer_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "packer_san")
    _build(tmp_path, ["g++", "-std=c++20", *SAN, "-I", os.path.join(ROOT, "include"), "-o", exe,
                      os.path.join(HERE, "cpp", "packer_test.cpp"), "-lpthread"])
    _run(exe)


@pytest.mark.skipif(not os.path.isdir(os.path.join(build_cpp.REF, "examples")),
                    reason="reference tree absent (GPU box)")
def test_reference_generated_stubs_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "calc_san")
    _build(tmp_path, ["g++", "-std=c++20", *SAN, "-Wno-unused-parameter", "-I", os.path.join(ROOT, "include"),
                      "-I", os.path.join(build_cpp.REF, "examples"), "-o", exe,
                      os.path.join(HERE, "cpp", "calculator_compat_test.cpp"), "-lpthread"])
    _run(exe, ok="calculator_compat_test: ok")
