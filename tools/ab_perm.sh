#!/bin/bash
# A/B timing of CSS permutation builds on the C5 shape: tools/ab_perm.sh TAG variant...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=$1; shift
mkdir -p gpurun_out/$T
for v in "$@"; do
  GDSCAN_LIB=tools/variants/$v/libgdscan.so POP=40 NCH=1 RUNS=1000 TRES=10 STEPS=3 timeout -k 10 120 python tools/css_time.py >> gpurun_out/$T/$v.txt 2>&1 || exit 1
done
