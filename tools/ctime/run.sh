#!/bin/bash
# Time the device compile of individual arithmetic pieces (tools/ctime/common.h) in parallel.
# Usage: tools/ctime/run.sh [PIECE ...]   (default: QMUL DEC FMUL ML FE)
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=/tmp/ctime
mkdir -p "$OUT"
PIECES=${*:-QMUL DEC FMUL ML FE}
for t in $PIECES; do
  (
    /usr/bin/time -f "$t %e s" timeout 600 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 \
      -D T_$t -I"$ROOT/include" -I"$ROOT/hbbft_amd/csrc" --cuda-device-only -x hip \
      -c "$ROOT/tools/ctime/common.h" -o "$OUT/$t.o" -Rpass-analysis=kernel-resource-usage \
      > "$OUT/$t.log" 2>&1
    tail -1 "$OUT/$t.log"
  ) &
done
wait
