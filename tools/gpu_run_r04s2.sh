# Round 4: kernel breakdown of the short single-string unpack (0-16 / 0-32 B).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04s2_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_paths.py --only string_0-16 --no-stream --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/r04s2.log 2>&1 || exit 2
