#!/bin/bash
# FET scan pipeline diagnostics: chromosome groups (GD_GROUPS) and the draw-free build
set -o pipefail
T=${1:-fg}
mkdir -p gpurun_out/$T
for g in 1 2 4 8; do
  GD_GROUPS=$g timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/$T/g$g.json 2> gpurun_out/$T/g$g.err || exit 1
done
for v in "$@"; do
  [ "$v" = "$T" ] && continue
  GDSCAN_LIB=tools/variants/$v/libgdscan.so timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/$T/$v.json 2> gpurun_out/$T/$v.err || exit 1
done
