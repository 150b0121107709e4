# Round 4: enveloped TILE unpack (Calculator rows): record kernel tile depth K
# and record vs generic kernels, interleaved A/B over build_ab/*.so.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_multi.sh 2 square_ add_request subtract two_numbers || exit 1
cp gpurun_out/ab.log gpurun_out/r04h_rec_ab.log
