set -o pipefail
mkdir -p gpurun_out
for t in 1,4,0 1,1,3 1,1,2 1,2,3 1,2,2 1,1,1 1,4,3 1,8,3; do
  timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --no-verify --tune $t >> gpurun_out/tune.log 2>&1 || exit 1
done
for t in 1,1,3 1,4,0 1,1,2; do
  timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --no-verify --tune $t >> gpurun_out/tune.log 2>&1 || exit 1
done
