# final tree check: every GPU test, then smoke
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 60 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03.log 2>&1
