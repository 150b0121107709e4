bash tools/gpu_prof_rows.sh "r05 now nozm" "multiple_primitives_zeros_4M zh4_straddle_heavy_4M zh4_straddle_heavy_long_256K string_0-16_8M" r06f || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_stream_r06f.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_stream_r06f.log
