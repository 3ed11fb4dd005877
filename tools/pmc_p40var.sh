#!/bin/bash
# VALU of the CSS kernels for phase-skip builds on the C3 shape: tools/pmc_p40var.sh TAG variant...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=$1; shift
for v in "$@"; do
  mkdir -p gpurun_out/$T/$v
  GDSCAN_LIB=tools/variants/$v/libgdscan.so POP=20 NCH=20 STEPS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
      -d gpurun_out/$T/$v/pmc -o run --output-format csv -- python3 tools/css_time.py > gpurun_out/$T/$v/out.txt 2> gpurun_out/$T/$v/err.txt || exit 1
done
