#!/bin/bash
# LDS and VALU activity of every kernel of one bench pass (FET + CSS legs): tools/pmc_lds.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-pmclds}
mkdir -p gpurun_out/$T
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
    SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d gpurun_out/$T/pmc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --css-steps 1 \
    --no-extra > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err
