#!/bin/bash
# VALU instruction count of the FET scan kernels for a library build ($1 = libgdscan.so, $2 = tag)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$2
GDSCAN_LIB=$1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
    -d gpurun_out/$2/pmc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-css --no-extra \
    > gpurun_out/$2/b.json 2> gpurun_out/$2/b.err
