mkdir -p gpurun_out
for m in plain pair3 pair2; do
  HBTC_CHECK_MODE=$m timeout -k 10 150 python -u bench.py --no-cpu --no-extra --steps 10 > gpurun_out/b11_$m.json 2> gpurun_out/b11_$m.err || exit $?
done
