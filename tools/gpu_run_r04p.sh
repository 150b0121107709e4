# Round 4: record-tile unpack without the chars image (SRPC_RTU_DIRECT=1,
# lane-per-record copies) vs with; also for short records (var_kernel 2).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SRPC_RTU_DIRECT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tiled.py -k "strings or tiled or table" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04p_tests_direct.log 2>&1 || exit 1
for r in 1 2; do
  for F in two_str string_0-16 string_0-32 str0-64; do
    timeout -k 10 300 python3 tools/bench_paths.py --only $F --reps 10 --var-kernel 1,2 > gpurun_out/r04p_img_${F}_$r.log 2>&1 || exit 2
    SRPC_RTU_DIRECT=1 timeout -k 10 300 python3 tools/bench_paths.py --only $F --reps 10 --var-kernel 1,2 > gpurun_out/r04p_direct_${F}_$r.log 2>&1 || exit 3
  done
done
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 --only string > gpurun_out/r04p_stream.log 2>&1 || exit 4
