# Interleaved A/B of build_ab/*.so over several bench_paths filters (one box).
# usage: bash tools/ab_multi.sh ROUNDS FILTER [FILTER ...]   -> gpurun_out/ab.log
set -o pipefail
mkdir -p gpurun_out
R=$1
shift
: > gpurun_out/ab.log
for r in $(seq 1 "$R"); do
  for F in "$@"; do
    for so in build_ab/*.so; do
      echo "== $(basename "$so" .so) round $r $F" >> gpurun_out/ab.log
      SRPC_GPU_LIB=$so timeout -k 10 300 python3 tools/bench_paths.py --only "$F" --reps 10 $AB_ARGS 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/ab.log || exit 1
    done
  done
done
