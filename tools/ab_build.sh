# Build A/B libraries for tools/ab_multi.sh: build_ab/a_<rev>.so from git REV's
# csrc (default HEAD) and build_ab/b_work.so from the working tree.
# usage: bash tools/ab_build.sh [REV]
set -e
REV=${1:-HEAD}
rm -rf build_ab /tmp/ab_src && mkdir -p build_ab /tmp/ab_src
git archive "$REV" srpc_amd/csrc include | tar -x -C /tmp/ab_src
python3 - "$REV" <<'PY'
import sys
from srpc_amd import build
rev = sys.argv[1].replace("/", "_")
print(build.build(out=f"build_ab/a_{rev}.so", srcdir="/tmp/ab_src/srpc_amd/csrc"))
print(build.build(out="build_ab/b_work.so", force=True))
PY
