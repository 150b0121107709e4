"""Build the C++ API-mirror test programs in tests/cpp/ (host code only)."""
from __future__ import annotations

import glob
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "_bin")


def build_all() -> list[str]:
    built = []
    for src in sorted(glob.glob(os.path.join(HERE, "*.cpp"))):
        built.append(build_one(src))
    return built


def build_one(src: str) -> str:
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, os.path.splitext(os.path.basename(src))[0])
    if os.path.exists(exe) and os.path.getmtime(exe) > max(
            os.path.getmtime(p) for p in [src] + glob.glob(os.path.join(ROOT, "include", "**", "*"),
                                                           recursive=True) if os.path.isfile(p)):
        return exe
    cmd = ["g++", "-std=c++20", "-O2", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"),
           "-o", exe, src, "-ldl", "-lpthread"]
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError(f"building {src} failed:\n{out.stdout}{out.stderr}")
    return exe
