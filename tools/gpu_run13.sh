# lane-count variants (HBTC_LIB_PATH): C3 slices
mkdir -p gpurun_out
for v in L5 L6; do
  export HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so
  for c in 125 250 1000; do
    timeout -k 10 120 python -u bench.py --no-cpu --no-extra --steps 12 --cts $c > gpurun_out/b13_${v}_$c.json 2> gpurun_out/b13_${v}_$c.err || exit $?
  done
done
