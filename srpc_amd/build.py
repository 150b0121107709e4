"""Build the in-tree HIP library ``srpc_amd/libsrpc_gpu.so`` for gfx950.

``python -m srpc_amd.build`` (or ``__graft_entry__.build()``) compiles
``srpc_amd/csrc/*.hip`` with hipcc into one shared library exporting the C ABI
of ``include/srpc_gpu.h``.  The .so stays in the source tree (git-ignored) so it
travels to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SO = os.path.join(PKG, "libsrpc_gpu.so")
ARCH = os.environ.get("SRPC_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: cannot build srpc_amd/libsrpc_gpu.so")


def sources() -> list[str]:
    return sorted(glob.glob(os.path.join(PKG, "csrc", "*.hip")))


def needs_build() -> bool:
    if not os.path.exists(SO):
        return True
    t = os.path.getmtime(SO)
    deps = sources() + glob.glob(os.path.join(PKG, "csrc", "*.h")) + [
        os.path.join(ROOT, "include", "srpc_gpu.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, out: str | None = None, srcdir: str | None = None,
          defines: tuple[str, ...] = ()) -> str:
    """Compile csrc/*.hip into SO (or `out`, from `srcdir`, with -D`defines`: A/B builds)."""
    if out is None and not force and not needs_build():
        return SO
    target = out or SO
    src = sorted(glob.glob(os.path.join(srcdir, "*.hip"))) if srcdir else sources()
    inc = srcdir or os.path.join(PKG, "csrc")
    tmp = target + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-command-line-argument",
           "-I", os.path.join(ROOT, "include"), "-I", inc] + [f"-D{d}" for d in defines] + ["-o", tmp] + src + [
           "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + out.stdout + out.stderr)
    os.replace(tmp, target)
    return target


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
