# VAR unpack: fused per-call resets -- string parity + stream tests, then A/B against HEAD
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "strings or schema_at or multi" > gpurun_out/t_var.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_golden.py > gpurun_out/t_stream.log 2>&1 && \
timeout -k 10 600 bash tools/ab_run.sh str 3
