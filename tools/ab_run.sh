# Interleaved A/B of the build_ab/*.so variants on one box: bench_paths for
# each variant, R rounds (A B A B ...).  usage: bash tools/ab_run.sh FILTER [ROUNDS] [bench_paths args]
set -o pipefail
mkdir -p gpurun_out
F=${1:-str}
R=${2:-2}
X=${3:-}
: > gpurun_out/ab.log
for r in $(seq 1 "$R"); do
  for so in build_ab/*.so; do
    echo "== $(basename "$so" .so) round $r" >> gpurun_out/ab.log
    SRPC_GPU_LIB=$so timeout -k 10 300 python3 tools/bench_paths.py --only "$F" --reps 10 $X 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/ab.log || exit 1
  done
done
