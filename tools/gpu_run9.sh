# kernel traces of the C3 bench for library variants (HBTC_LIB_PATH), per-kernel stats
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then unset HBTC_LIB_PATH; else export HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt9_$v -o kt -- python3 bench.py --no-cpu --no-extra --steps 3 --warmup 1 > gpurun_out/kt9_$v.log 2>&1 || exit $?
done
