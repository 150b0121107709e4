set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit 1
for b in 65536 262144 1048576; do
  timeout -k 10 120 ./tools/e2e_square --mode gpu --n 1048576 --batch $b --port 18400 >> gpurun_out/e2e.log 2>&1 || exit 2
done
timeout -k 10 120 ./tools/e2e_square --mode cpu --n 1048576 --port 18401 >> gpurun_out/e2e.log 2>&1 || exit 3
