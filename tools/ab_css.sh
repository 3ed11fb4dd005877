#!/bin/bash
# A/B timing of CSS library builds: [POPS="20 40"] tools/ab_css.sh TAG variant... (tools/variants/<v>/libgdscan.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=$1; shift
mkdir -p gpurun_out/$T
for v in "$@"; do
  for pop in ${POPS:-20 40}; do
    NCH=$([ $pop -le 20 ] && echo 20 || echo 4)
    GDSCAN_LIB=tools/variants/$v/libgdscan.so POP=$pop NCH=$NCH STEPS=5 timeout -k 10 120 python tools/css_time.py >> gpurun_out/$T/$v.txt 2>&1 || exit 1
  done
done
