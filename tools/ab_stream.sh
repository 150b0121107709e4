# Interleaved A/B of the build_ab/*.so variants on the stream decode: the
# stream_bench rows and bench_paths' VAR rows (its stream column), R rounds.
# usage: bash tools/ab_stream.sh [ROUNDS]
set -o pipefail
mkdir -p gpurun_out
R=${1:-2}
: > gpurun_out/ab_stream.log
for r in $(seq 1 "$R"); do
  for so in build_ab/*.so; do
    v=$(basename "$so" .so)
    SRPC_GPU_LIB=$so timeout -k 10 300 python3 tools/stream_bench.py --reps 10 2>/dev/null | grep -v amdgpu.ids | sed "s/^/$v sb /" >> gpurun_out/ab_stream.log || exit 1
    SRPC_GPU_LIB=$so timeout -k 10 300 python3 tools/bench_paths.py --only str --reps 10 2>/dev/null | grep -v amdgpu.ids | sed "s/^/$v bp /" >> gpurun_out/ab_stream.log || exit 1
  done
done
