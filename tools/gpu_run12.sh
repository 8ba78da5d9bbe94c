# lane-count / preparation-placement variants: C3 slices and C2
mkdir -p gpurun_out
for v in L4 L4P L3P; do
  export HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so
  for c in 125 1000; do
    timeout -k 10 120 python -u bench.py --no-cpu --no-extra --steps 10 --cts $c > gpurun_out/b12_${v}_$c.json 2> gpurun_out/b12_${v}_$c.err || exit $?
  done
  timeout -k 10 200 python -u bench_configs.py --configs c2 > gpurun_out/b12_${v}_c2.json 2> gpurun_out/b12_${v}_c2.err || exit $?
done
