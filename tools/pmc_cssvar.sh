#!/bin/bash
# SQ_INSTS_VALU of the CSS kernels for several library builds: tools/pmc_cssvar.sh TAG lib...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=$1; shift
for L in "$@"; do
  N=$(basename $(dirname $L))
  mkdir -p gpurun_out/$T/$N
  GDSCAN_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS \
      -d gpurun_out/$T/$N/pmc -o run --output-format csv -- python3 tools/css_time.py \
      > gpurun_out/$T/$N/out.txt 2> gpurun_out/$T/$N/err.txt || exit 1
done
