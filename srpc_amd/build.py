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


def _objdir(target: str) -> str:
    return os.path.join(os.path.dirname(target), "build", os.path.basename(target) + ".objs")


def build(force: bool = False, verbose: bool = False, out: str | None = None, srcdir: str | None = None,
          defines: tuple[str, ...] = ()) -> str:
    """Compile csrc/*.hip into SO (or `out`, from `srcdir`, with -D`defines`: A/B builds).

    One hipcc per source file, in parallel, into objects kept beside the
    target (build/<so>.objs/), then one link: a rebuild after editing one
    file recompiles that file only (headers, the flags or `force` recompile
    all).  Each file is its own code object (no -fgpu-rdc: no kernel calls a
    device function of another file)."""
    if out is None and not force and not needs_build():
        return SO
    from concurrent.futures import ThreadPoolExecutor

    target = out or SO
    src = sorted(glob.glob(os.path.join(srcdir, "*.hip"))) if srcdir else sources()
    inc = srcdir or os.path.join(PKG, "csrc")
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-command-line-argument",
             "-I", os.path.join(ROOT, "include"), "-I", inc] + [f"-D{d}" for d in defines]
    objdir = _objdir(target)
    os.makedirs(objdir, exist_ok=True)
    stamp = os.path.join(objdir, "flags.txt")
    same_flags = os.path.exists(stamp) and open(stamp).read() == " ".join(flags)
    headers = glob.glob(os.path.join(inc, "*.h")) + [os.path.join(ROOT, "include", "srpc_gpu.h")]
    newest_header = max(os.path.getmtime(h) for h in headers if os.path.exists(h))

    def compile_one(path: str) -> str:
        obj = os.path.join(objdir, os.path.basename(path) + ".o")
        if (not force and same_flags and os.path.exists(obj)
                and os.path.getmtime(obj) > max(os.path.getmtime(path), newest_header)):
            return ""
        cmd = [hipcc()] + flags + ["-c", "-o", obj + ".tmp", path]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            return f"hipcc failed on {path}:\n{r.stdout}{r.stderr}"
        os.replace(obj + ".tmp", obj)
        return ""

    jobs = max(1, min(len(src), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 4), 16))
    with ThreadPoolExecutor(jobs) as ex:
        errs = [e for e in ex.map(compile_one, src) if e]
    if errs:
        raise RuntimeError("\n".join(errs))
    with open(stamp, "w") as f:
        f.write(" ".join(flags))
    objs = [os.path.join(objdir, os.path.basename(p) + ".o") for p in src]
    tmp = target + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", tmp] + objs + [
           "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc link failed:\n" + r.stdout + r.stderr)
    os.replace(tmp, target)
    return target


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
