mkdir -p gpurun_out
for v in NO_SUBGROUP NO_SMUL NO_PKMUL; do
  HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so timeout -k 10 120 python -u bench.py --no-cpu --no-extra --steps 3 > gpurun_out/v8_$v.json 2> gpurun_out/v8_$v.err
  rc=$?; if [ $rc -gt 1 ]; then exit $rc; fi
done
exit 0
