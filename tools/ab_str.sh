set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.log
for r in 1 2; do
  for so in build_ab/*.so; do
    echo "== $(basename "$so" .so) round $r" >> gpurun_out/ab.log
    SRPC_GPU_LIB=$so timeout -k 10 200 python3 tools/bench_paths.py --only str --reps 10 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/ab.log || exit 1
  done
done
