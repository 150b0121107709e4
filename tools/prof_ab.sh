# Per-kernel durations (rocprofv3 --kernel-trace) of tools/bench_paths.py for
# every build_ab/*.so variant.  usage (through gpurun): bash tools/prof_ab.sh FILTER [bench_paths args]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F=${1:-str}
X=${2:-}
: > gpurun_out/prof_ab.txt
for so in build_ab/*.so; do
  v=$(basename "$so" .so)
  SRPC_GPU_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_ab_$v -o run --output-format csv -- python3 tools/bench_paths.py --only "$F" --reps 5 $X > gpurun_out/prof_ab_$v.log 2>&1 || exit 1
  echo "== $v" >> gpurun_out/prof_ab.txt
  python3 tools/kernel_table.py gpurun_out/prof_ab_$v/run_kernel_trace.csv >> gpurun_out/prof_ab.txt || exit 2
done
