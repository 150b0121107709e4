# Round 4: the same rows under the round-3 tree, the first round-4 AoS build
# and the working tree, interleaved on one box (box or code?).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_multi.sh 2 quad_tile all_kinds_aos || exit 1
cp gpurun_out/ab.log gpurun_out/r04s_ab.log
