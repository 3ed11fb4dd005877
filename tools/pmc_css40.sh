#!/bin/bash
# SQ counters of the CSS kernels on the C3 shape (20+20) for a library build: tools/pmc_css40.sh TAG [lib]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-pmc40}
mkdir -p gpurun_out/$T
GDSCAN_LIB=${2:-} POP=20 NCH=20 STEPS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d gpurun_out/$T/pmc -o run --output-format csv -- python3 tools/css_time.py > gpurun_out/$T/out.txt 2> gpurun_out/$T/err.txt
