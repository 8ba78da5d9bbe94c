mkdir -p gpurun_out
for c in 125 250 1000; do
  timeout -k 10 120 python -u bench.py --no-cpu --no-extra --steps 10 --cts $c > gpurun_out/b7_${c}.json 2> gpurun_out/b7_${c}.err || exit $?
done
timeout -k 10 200 python -u bench_configs.py --configs c2 > gpurun_out/b7_c2.json 2> gpurun_out/b7_c2.err || exit $?
