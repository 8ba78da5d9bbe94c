#!/bin/bash
# r05 session 19: the co-Z chain build reordered (XP dropped after two steps, 22 rescaled entries):
# RLC parity, C3 A/B against the round's earlier build (old), then the headline profile (kernel
# trace + PMC passes, tools/profile.sh) of this build; and the SignatureShare kernels with the
# product inlined.  Outcome: C3 71.9 vs 71.6 ms (old), kept; the sginl C4 run printed nothing
# for 180 s and was stopped by gpurun (variant dropped); the profile step did not run (run20.sh).
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run19
mkdir -p $O
step 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py > $O/parity.log 2>&1
for v in old base old base old base; do
  HBTC_LIB_PATH=$(lib $v) step 150 python -u bench.py --no-cpu --no-extra > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
# the SignatureShare kernels with the Fq product inlined (sginl) instead of the shared subroutine:
# k_sig_decode's loops then run without scratch (tools/isa_loops.py); C4 and C2
for v in base sginl base sginl; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_$v.$RANDOM.json 2>> $O/c4.err
done
for v in base sginl; do
  HBTC_LIB_PATH=$(lib $v) step 200 python -u bench_configs.py --configs c2 --no-cpu > $O/c2_$v.json 2>> $O/c2.err
done
rm -rf gpurun_out/prof_bench_1000ct_128b
step 900 bash tools/profile.sh bench_1000ct_128b
echo all-done >&2
