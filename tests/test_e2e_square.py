"""BASELINE.json configs[4]: Calculator.square end to end over 127.0.0.1 with
the server decoding, squaring and encoding whole batches on the GPU
(include/srpc/gpu_server.hpp).  Every response is checked by the client with
unpack_response<Number>; the unframed response stream of the full 1M run must
hash to the reference digest (tests/golden/manifest.json)."""
import hashlib
import json
import os
import subprocess

import pytest

from tools import build_tools

pytestmark = pytest.mark.gpu


def _run(*args, timeout=300):
    exe = build_tools.build("e2e_square")
    out = subprocess.run([exe, *args], capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stdout + out.stderr
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_e2e_square_gpu_batches_small():
    r = _run("--mode", "gpu", "--n", "70001", "--batch", "16384", "--port", "18301")
    assert r["ok"] and r["gpu"]["fallback_requests"] == 0 and r["gpu"]["batches"] >= 5


def test_e2e_square_fallback_on_foreign_frame():
    r = _run("--mode", "gpu", "--n", "50000", "--batch", "8192", "--port", "18302", "--poison", "12345")
    assert r["ok"] and r["gpu"]["fallback_requests"] >= 1


def test_e2e_square_fallback_on_foreign_frame_of_other_length():
    """A foreign frame 7 bytes longer moves every later frame off the 57-byte
    grid: the rest of its batch and the bytes already read for the next batch
    are answered on the CPU, after which batching resumes."""
    r = _run("--mode", "gpu", "--n", "50000", "--batch", "8192", "--port", "18304", "--poison", "20000",
             "--poison-method", "Calculator_servicer::square_v2")
    assert r["ok"] and r["gpu"]["fallback_requests"] >= 1


@pytest.mark.slow
def test_e2e_square_1M_reference_digest(manifest, tmp_path):
    dump = str(tmp_path / "resp.bin")
    r = _run("--mode", "gpu", "--n", str(1 << 20), "--port", "18303", "--dump", dump)
    assert r["ok"]
    with open(dump, "rb") as f:
        digest = hashlib.sha256(f.read()).hexdigest()
    assert digest == manifest["streams"]["square_responses_1M"]["sha256"]
