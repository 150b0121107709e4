# Round 4: stream decoder (sdx.hip) tests + whole-call bench + per-kernel split
# (rocprofv3 kernel trace) on three rows; TILE unpack A/B on the fixed rows.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_tiled.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04c_stream_new.log 2>&1 || exit 2
for F in multiple_primitives_str0-64 two_str_request zh4_zero_heavy_4M; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04c_sprof_$F -o run --output-format csv -- python3 tools/stream_bench.py --reps 5 --only $F > gpurun_out/r04c_sprof_$F.log 2>&1 || exit 3
done
timeout -k 10 600 bash tools/ab_run.sh B_16M 2 || exit 4
cp gpurun_out/ab.log gpurun_out/r04c_tile_ab.log
