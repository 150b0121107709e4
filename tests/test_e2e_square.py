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


def _run(*args, timeout=300, slots=None):
    exe = build_tools.build("e2e_square")
    env = dict(os.environ)
    if slots is not None:
        env["SRPC_SERVER_SLOTS"] = slots
    out = subprocess.run([exe, *args], capture_output=True, text=True, timeout=timeout, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    return json.loads(out.stdout.strip().splitlines()[-1])


def _served(r, n):
    g = r["gpu"]
    assert r["ok"], r
    assert g["gpu_requests"] + g["fallback_requests"] == n, r
    return g


def test_e2e_square_gpu_batches_small():
    r = _run("--mode", "gpu", "--n", "70001", "--batch", "16384", "--port", "18301")
    g = _served(r, 70001)
    assert g["fallback_requests"] == 0 and g["batches"] >= 5 and g["mixed_batches"] == 0


def test_e2e_square_only_the_foreign_frame_leaves_the_gpu():
    r = _run("--mode", "gpu", "--n", "50000", "--batch", "8192", "--port", "18302", "--poison", "12345")
    assert _served(r, 50000)["fallback_requests"] == 1


def test_e2e_square_foreign_frame_of_other_length():
    """A foreign frame 7 bytes longer is still one frame: the CPU walks the
    BE32 lengths, so every later frame stays on the GPU."""
    r = _run("--mode", "gpu", "--n", "50000", "--batch", "8192", "--port", "18304", "--poison", "20000",
             "--poison-method", "Calculator_servicer::square_v2")
    assert _served(r, 50000)["fallback_requests"] == 1


def test_e2e_square_poison_at_index_0_of_a_256k_batch():
    n = 1 << 18
    r = _run("--mode", "gpu", "--n", str(n), "--batch", str(n), "--port", "18305", "--poison", "0")
    g = _served(r, n)
    assert g["fallback_requests"] == 1 and g["gpu_requests"] == n - 1
    print(json.dumps(r))


def test_e2e_one_percent_foreign_traffic():
    """1 % divide requests (a method the GPU server does not have) among
    squares: exactly those go to the CPU server, answered in their places."""
    n = 200_000
    r = _run("--mode", "gpu", "--n", str(n), "--batch", "65536", "--port", "18306", "--foreign", "0.01")
    g = _served(r, n)
    assert 1500 < r["traffic"]["divide"] < 2500
    assert g["fallback_requests"] == r["traffic"]["divide"]
    print(json.dumps(r))


def test_e2e_mixed_methods_all_on_the_gpu():
    """square + add / subtract / multiply (two frame lengths) in one stream,
    all four registered on the GPU: bucketed per method, nothing on the CPU."""
    n = 120_000
    r = _run("--mode", "gpu", "--n", str(n), "--batch", "32768", "--port", "18307", "--mix", "0.3",
             "--gpu-methods", "all")
    g = _served(r, n)
    assert g["fallback_requests"] == 0 and g["mixed_batches"] >= 1
    assert min(r["traffic"][m] for m in ("add", "subtract", "multiply")) > 5000


def test_e2e_mixed_methods_some_on_the_cpu():
    n = 60_000
    r = _run("--mode", "gpu", "--n", str(n), "--batch", "16384", "--port", "18308", "--mix", "0.2",
             "--foreign", "0.05", "--poison", "0,17,59999")
    g = _served(r, n)
    t = r["traffic"]
    assert g["fallback_requests"] == t["add"] + t["subtract"] + t["multiply"] + t["divide"] + t["poison"]
    assert t["poison"] == 3


@pytest.mark.parametrize("slots", ["1", "2"])
def test_e2e_one_or_two_batches_in_flight(slots):
    """The server's two staging slots (a batch's kernels and copies run while
    the next batch is received; SRPC_SERVER_SLOTS=1: one at a time): the same
    responses either way, foreign frames and poison included."""
    n = 90_000
    r = _run("--mode", "gpu", "--n", str(n), "--batch", "8192", "--port", str(18320 + int(slots)), "--mix",
             "0.2", "--foreign", "0.02", "--poison", "0,8191,8192,89999", "--gpu-methods", "all", slots=slots)
    g = _served(r, n)
    t = r["traffic"]
    assert g["fallback_requests"] == t["divide"] + t["poison"] and t["poison"] == 4
    assert g["batches"] >= 10


@pytest.mark.parametrize("at", [0, 3000])
def test_e2e_frame_larger_than_the_batch_buffer(at):
    """A frame longer than the whole receive buffer is read on its own and
    answered on the CPU; the connection carries on."""
    n = 20_000
    r = _run("--mode", "gpu", "--n", str(n), "--batch", "4096", "--port", str(18309 + at % 7), "--oversize",
             str(at), "--poison", "5000")
    g = _served(r, n)
    assert g["oversize_requests"] == 1 and g["fallback_requests"] == 2


@pytest.mark.slow
def test_e2e_square_1M_reference_digest(manifest, tmp_path):
    dump = str(tmp_path / "resp.bin")
    r = _run("--mode", "gpu", "--n", str(1 << 20), "--port", "18303", "--dump", dump)
    assert r["ok"]
    with open(dump, "rb") as f:
        digest = hashlib.sha256(f.read()).hexdigest()
    assert digest == manifest["streams"]["square_responses_1M"]["sha256"]


# ---- a string-bodied method (Echo_servicer::echo over multiple_primitives) ----
def test_e2e_echo_string_method_all_on_the_gpu():
    """Every request carries a string: classified, gathered with a record
    index, unpacked, echoed, packed and framed on the GPU; the client checks
    each answer byte for byte against the scalar packer's."""
    n = 100_000
    r = _run("--mode", "gpu", "--n", str(n), "--batch", "16384", "--port", "18321", "--echo", "1",
             "--gpu-methods", "square,echo")
    g = _served(r, n)
    assert g["fallback_requests"] == 0 and g["gpu_requests"] == n and r["traffic"]["echo"] == n


def test_e2e_echo_reference_digest(manifest, tmp_path):
    """The unframed response stream of 200,000 echo requests equals the
    reference server's (tests/golden/make_golden.py ref_server_echo)."""
    want = manifest["streams"]["echo_responses"]
    dump = str(tmp_path / "echo.bin")
    r = _run("--mode", "gpu", "--n", str(want["records"]), "--batch", "65536", "--port", "18322", "--echo", "1",
             "--gpu-methods", "echo", "--dump", dump)
    assert _served(r, want["records"])["fallback_requests"] == 0
    with open(dump, "rb") as f:
        b = f.read()
    assert len(b) == want["bytes"] and hashlib.sha256(b).hexdigest() == want["sha256"]


def test_e2e_echo_mixed_with_fixed_methods_and_foreign_traffic():
    """Echo, square, add/subtract/multiply on the GPU in one stream with 1 %
    divide and three poisoned frames on the CPU: answers in request order."""
    n = 120_000
    r = _run("--mode", "gpu", "--n", str(n), "--batch", "32768", "--port", "18323", "--echo", "0.3", "--mix", "0.2",
             "--foreign", "0.01", "--poison", "0,7,119999", "--gpu-methods", "all,echo")
    g = _served(r, n)
    t = r["traffic"]
    assert t["echo"] > 30_000 and g["fallback_requests"] == t["divide"] + t["poison"]
    assert g["mixed_batches"] >= 1


def test_e2e_echo_on_the_cpu_when_not_registered():
    n = 30_000
    r = _run("--mode", "gpu", "--n", str(n), "--batch", "8192", "--port", "18324", "--echo", "0.25")
    g = _served(r, n)
    assert g["fallback_requests"] == r["traffic"]["echo"] > 5000


def test_e2e_echo_responses_past_max_response_chars():
    """Echo answers (0..41 chars each) into response columns sized for 8
    chars per request on average: a full batch's answers do not fit, so its
    echo frames are answered by the CPU server in their places (nothing reads
    past the columns, the connection keeps serving); square stays on the GPU
    and every answer is checked by the client."""
    n = 40_000
    r = _run("--mode", "gpu", "--n", str(n), "--batch", "8192", "--port", "18325", "--echo", "0.8",
             "--gpu-methods", "square,echo", "--max-resp-chars", "8")
    g = _served(r, n)
    assert g["overflow_batches"] >= 1
    assert 0 < g["fallback_requests"] <= r["traffic"]["echo"]
    assert g["gpu_requests"] + g["fallback_requests"] == n
