"""Build the C++ API-mirror test programs in tests/cpp/ (host code only)."""
from __future__ import annotations

import glob
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "_bin")


REF = "/root/reference"
ROCM = "/opt/rocm"


def needs(src: str) -> set[str]:
    """`// needs: reference, gpu` on the first line of a test source."""
    first = open(src).readline()
    if first.startswith("// needs:"):
        return {w.strip() for w in first.split(":", 1)[1].split(",")}
    return set()


def exe_path(src: str) -> str:
    return os.path.join(OUT, os.path.splitext(os.path.basename(src))[0])


def build_all() -> list[str]:
    built = []
    for src in sorted(glob.glob(os.path.join(HERE, "*.cpp"))):
        if "reference" in needs(src) and not os.path.isdir(os.path.join(REF, "examples")):
            continue  # the reference tree only exists in the build container
        built.append(build_one(src))
    return built


BATCHGEN_CONTRACT = os.path.join(HERE, "batchgen_example.contract")
BATCHGEN_HEADER = os.path.join(OUT, "batchgen_example_batch.hpp")


def generate_batch_header() -> str:
    """srpc_amd.batchgen over the example contract (message structs included)."""
    import sys
    sys.path.insert(0, ROOT)
    from srpc_amd import batchgen
    os.makedirs(OUT, exist_ok=True)
    text = batchgen.generate(batchgen.parse(open(BATCHGEN_CONTRACT).read()), "batchgen_example.contract",
                             messages=True)
    if not os.path.exists(BATCHGEN_HEADER) or open(BATCHGEN_HEADER).read() != text:
        with open(BATCHGEN_HEADER, "w") as f:
            f.write(text)
    return BATCHGEN_HEADER


def build_one(src: str) -> str:
    os.makedirs(OUT, exist_ok=True)
    exe = exe_path(src)
    req = needs(src)
    deps = [src] + glob.glob(os.path.join(ROOT, "include", "**", "*"), recursive=True) + \
        glob.glob(os.path.join(HERE, "*.hpp"))
    if "batchgen" in req:
        deps.append(generate_batch_header())
    if os.path.exists(exe) and os.path.getmtime(exe) > max(os.path.getmtime(p) for p in deps if os.path.isfile(p)):
        return exe
    cmd = ["g++", "-std=c++20", "-O2", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"), "-I", OUT,
           "-o", exe, src]
    if "reference" in req:
        cmd += ["-I", os.path.join(REF, "examples"), "-Wno-unused-parameter"]
    if "gpu" in req:
        pkg = os.path.join(ROOT, "srpc_amd")
        cmd += ["-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROCM, "include"), "-L", pkg, "-lsrpc_gpu",
                f"-Wl,-rpath,{pkg}", "-L", os.path.join(ROCM, "lib"), "-lamdhip64",
                f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"]
    cmd += ["-ldl", "-lpthread"]
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError(f"building {src} failed:\n{out.stdout}{out.stderr}")
    return exe
