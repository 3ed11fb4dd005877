#!/bin/bash
# LDS / VALU counters of the CSS permutation kernel on the C5 shape (1 chromosome, 40+40,
# 1000 permutations), for the in-tree library and any variants: tools/pmc_perm.sh TAG [variant...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-pmcperm}; shift
mkdir -p gpurun_out/$T
export POP=40 NCH=1 RUNS=1000 TRES=10 STEPS=1
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/$T/main -o run --output-format csv -- \
    python3 tools/css_time.py > gpurun_out/$T/main.txt 2>&1 || exit 1
for v in "$@"; do
  GDSCAN_LIB=tools/variants/$v/libgdscan.so timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/$T/$v -o run \
      --output-format csv -- python3 tools/css_time.py > gpurun_out/$T/$v.txt 2>&1 || exit 1
done
