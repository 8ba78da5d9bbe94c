mkdir -p gpurun_out
for v in base siginl; do
  if [ $v = base ]; then unset HBTC_LIB_PATH; else export HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so; fi
  timeout -k 10 300 python -u bench_configs.py --configs c4 > gpurun_out/b10_$v.json 2> gpurun_out/b10_$v.err || exit $?
done
