# Kernel split (rocprofv3 --kernel-trace) of stream_bench rows for library
# builds in build_ab/: bash tools/gpu_prof_rows.sh "lib1 lib2" "row1 row2" TAG
set -o pipefail
libs=$1; rows=$2; tag=${3:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in $libs; do
  for row in $rows; do
    out=gpurun_out/prof_${tag}_${lib}_${row}
    SRPC_GPU_LIB=build_ab/$lib.so timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out -o run -- python3 -u tools/stream_bench.py --reps 3 --only $row > $out.log 2>&1 || exit 1
    f=$(find $out -name '*kernel_trace.csv' | head -1)
    echo "## $lib $row" >> gpurun_out/prof_${tag}.txt
    grep -E " us " $out.log >> gpurun_out/prof_${tag}.txt
    python3 tools/kernel_table.py $f >> gpurun_out/prof_${tag}.txt || exit 2
    rm -rf $out
  done
done
