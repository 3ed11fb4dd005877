#!/bin/bash
# A/B timing of libgdscan.so builds on the FET bench: tools/ab_fet.sh OUTDIR lib1 lib2 ...
set -o pipefail
O=$1; shift
mkdir -p $O
for L in "$@"; do
  T=$(basename $(dirname $L))
  for r in 1 2; do
    GDSCAN_LIB=$L timeout -k 10 100 python bench.py --no-cpu --no-css > $O/$T.$r.json 2> $O/$T.$r.err || exit 1
  done
done
