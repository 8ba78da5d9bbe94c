mkdir -p gpurun_out
for p in 0 1; do for c in 125 250 1000; do
  HBTC_COMB_PRIO=$p timeout -k 10 120 python -u bench.py --no-cpu --no-extra --steps 10 --cts $c > gpurun_out/b6_${c}_$p.json 2> gpurun_out/b6_${c}_$p.err || exit $?
done; done
