# round-3 late session: AoS fresh-object unpack (run vs staged), stream window rotation A/B, stream rows on HEAD+
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 200 python3 tools/bench_paths.py --reps 10 --only aos > gpurun_out/paths_aos.log 2>&1 && \
SRPC_AOS_FILL_STAGED=1 timeout -k 10 200 python3 tools/bench_paths.py --reps 10 --only aos > gpurun_out/paths_aos_staged.log 2>&1 && \
timeout -k 10 300 python3 tools/stream_bench.py --reps 10 > gpurun_out/stream_cur.log 2>&1 && \
timeout -k 10 600 bash tools/ab_run.sh str 2
