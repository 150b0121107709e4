# Round 4: stream decoder on long strings (0-1024 B): phases and kernel split.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SRPC_GPU_LIB=build_sx/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py --only 0-1024 > gpurun_out/r04i_phases.log 2>&1 || exit 3
F=string_0-1024
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04i_sprof_$F -o run --output-format csv -- python3 tools/stream_bench.py --reps 5 --only $F > gpurun_out/r04i_sprof_$F.log 2>&1 || exit 4
