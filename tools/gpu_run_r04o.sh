# Round 4: AoS layout kernels direct vs through LDS (SRPC_AOS_LAY_T=1);
# PMC of the stream decode and of the two-string rows (tiled unpack);
# decode copying long strings a wave per record.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_aos.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04o_stream.log 2>&1 || exit 11
SRPC_AOS_LAY_T=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_aos.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04o_tests_t.log 2>&1 || exit 2
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_paths.py --only all_kinds_aos --reps 10 > gpurun_out/r04o_aos_direct_$r.log 2>&1 || exit 3
  SRPC_AOS_LAY_T=1 timeout -k 10 300 python3 tools/bench_paths.py --only all_kinds_aos --reps 10 > gpurun_out/r04o_aos_t_$r.log 2>&1 || exit 4
done
PMC_TOOL=stream_bench.py bash tools/pmc_paths.sh r04o_stream str0-64 two_str || exit 5
bash tools/pmc_paths.sh r04o two_str || exit 6
