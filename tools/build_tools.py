"""Build the HIP tool programs in tools/ (config-5 end-to-end harness)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

TOOLS = {"e2e_square": "e2e_square.hip", "aos_bench": "aos_bench.hip",
         "capture_ring": "capture_ring.hip"}  # (plain HIP: the library is linked, not used)


def build(name: str = "e2e_square") -> str:
    from srpc_amd import build as lib
    lib.build()
    src = os.path.join(HERE, TOOLS[name])
    exe = os.path.join(HERE, name)
    deps = [src, lib.SO] + [os.path.join(ROOT, "include", "srpc", f)
                            for f in os.listdir(os.path.join(ROOT, "include", "srpc"))]
    if os.path.exists(exe) and os.path.getmtime(exe) > max(os.path.getmtime(d) for d in deps):
        return exe
    cmd = [lib.hipcc(), f"--offload-arch={lib.ARCH}", "-O3", "-std=c++20", "-Wno-unused-command-line-argument",
           "-I", os.path.join(ROOT, "include"), "-o", exe, src, "-L", os.path.join(ROOT, "srpc_amd"),
           "-lsrpc_gpu", "-Wl,-rpath,$ORIGIN/../srpc_amd", "-lpthread"]
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError(f"building {name} failed:\n{out.stdout}{out.stderr}")
    return exe


if __name__ == "__main__":
    print(build(sys.argv[1] if len(sys.argv) > 1 else "e2e_square"))
