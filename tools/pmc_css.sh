#!/bin/bash
# SQ instruction / LDS counters of one bench run (FET + CSS legs): tools/pmc_css.sh TAG [lib]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$1
GDSCAN_LIB=${2:-fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd/lib/libgdscan.so} \
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU \
    -d gpurun_out/$1/pmc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --css-steps 1 \
    > gpurun_out/$1/b.json 2> gpurun_out/$1/b.err
