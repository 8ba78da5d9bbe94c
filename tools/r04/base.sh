set -o pipefail
mkdir -p gpurun_out/r04base
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04base/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 > gpurun_out/r04base/bench.json 2> gpurun_out/r04base/bench.err &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --cts 125 --no-cpu --no-extra > gpurun_out/r04base/slice125.json 2> gpurun_out/r04base/slice125.err
