# Round 4: TILE gather/stepped-phase change vs the round-3 code paths
# (SRPC_TILE_GATHER_OLD), interleaved on one box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_multi.sh 2 quad_tile all_kinds_17B _request_ _response_ || exit 1
cp gpurun_out/ab.log gpurun_out/r04t_ab.log
