# Per-kernel durations of the VAR path cases of tools/bench_paths.py (one MI355X).
# usage (through gpurun): bash tools/prof_var.sh [filter]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F=${1:-str}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_var -o run --output-format csv -- python3 tools/bench_paths.py --only "$F" --reps 5 > gpurun_out/prof_var.log 2>&1 || exit 1
python3 tools/kernel_table.py gpurun_out/prof_var/run_kernel_trace.csv > gpurun_out/prof_var_table.txt || exit 2
