#!/bin/bash
# FET window-kernel profile: kernel stats + one SQ counter pass (instruction mix).
# usage (GPU box): tools/prof_fet.sh TAG
set -o pipefail
T=${1:-fet}
O=gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu --no-css > $O/ktrace_bench.json 2> $O/ktrace.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM \
    -d $O/pmc_sq -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-css > $O/pmc_sq.json 2> $O/pmc_sq.err
echo "prof_fet exit $?"
