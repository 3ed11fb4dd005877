#!/bin/bash
# One GPU-box profiling pass for a round: bench line, kernel trace + stats, and the
# HBM PMC counters (FETCH_SIZE and WRITE_SIZE in separate passes).  Every GPU step
# has its own time limit and the steps are chained with &&.
# usage: tools/profile_round.sh r02
set -o pipefail
R=${1:-r02}
O=gpurun_out/$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/ktrace_bench.json 2> $O/ktrace.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-css --no-extra > $O/pmc_fetch.json 2> $O/pmc_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-css --no-extra > $O/pmc_write.json 2> $O/pmc_write.err &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS -d $O/pmc_valu -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-css --no-extra > $O/pmc_valu.json 2> $O/pmc_valu.err &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $O/pmc_css_valu -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --css-steps 1 --no-extra > $O/pmc_css_valu.json 2> $O/pmc_css_valu.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_css_fetch -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --css-steps 1 --no-extra > $O/pmc_css.json 2> $O/pmc_css.err &&
POP=40 NCH=1 RUNS=1000 TRES=10 STEPS=1 timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_perm -o run \
    --output-format csv -- python3 tools/css_time.py > $O/pmc_perm.txt 2> $O/pmc_perm.err
echo "profile_round exit $?"
