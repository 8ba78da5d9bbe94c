mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "rlc or rank_slice or back_to_back or tracking or node or c3_full" > gpurun_out/t5.log 2>&1 || exit $?
for c in 125 250 500 1000; do
  timeout -k 10 120 python -u bench.py --no-cpu --no-extra --steps 10 --cts $c > gpurun_out/b5_$c.json 2> gpurun_out/b5_$c.err || exit $?
done
for m in plain pair3 pair2; do for c in 125 250; do
  HBTC_CHECK_MODE=$m timeout -k 10 120 python -u bench.py --no-cpu --no-extra --steps 10 --cts $c > gpurun_out/b5_${c}_$m.json 2> gpurun_out/b5_${c}_$m.err || exit $?
done; done
