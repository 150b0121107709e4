#!/usr/bin/env python3
"""Build A/B variants of libsrpc_gpu.so into build_ab/ (git-ignored, travels
to the GPU box): each variant is a git revision's csrc/ (or the working tree)
plus optional -D defines.  Run a tool against one with SRPC_GPU_LIB=<path>.

    python tools/ab_build.py base=HEAD new=WORKTREE [name=REV:DEFINE1,DEFINE2 ...]
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv):
    from srpc_amd import build
    out_dir = os.path.join(ROOT, "build_ab")
    os.makedirs(out_dir, exist_ok=True)
    for spec in argv:
        name, _, rest = spec.partition("=")
        rev, _, defs = rest.partition(":")
        defines = tuple(d for d in defs.split(",") if d)
        if rev == "WORKTREE":
            srcdir = os.path.join(ROOT, "srpc_amd", "csrc")
        else:
            srcdir = tempfile.mkdtemp(prefix=f"ab_{name}_")
            files = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", rev, "srpc_amd/csrc/"],
                                   capture_output=True, text=True, check=True).stdout.split()
            for f in files:
                data = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{f}"], capture_output=True,
                                      check=True).stdout
                with open(os.path.join(srcdir, os.path.basename(f)), "wb") as fh:
                    fh.write(data)
        path = build.build(out=os.path.join(out_dir, f"{name}.so"), srcdir=srcdir, defines=defines)
        print(name, path)


if __name__ == "__main__":
    main(sys.argv[1:])
