#!/bin/bash
# One GPU-box profiling pass (per round): the VALU microbenchmark (issue peak per op class),
# the bench line, kernel trace + stats, and PMC passes, each in a run of its own:
#   FET: FETCH_SIZE, WRITE_SIZE (HBM traffic), SQ issue counters of the scan kernels
#   CSS: SQ issue counters of the C3 (k_css_pack + k_css_mds_p40), C4 (k_css_mds_t80) and
#        C5 permutation (k_css_perm<80>) kernels
# Every GPU step has its own time limit; the steps are chained with &&.
# The CSS distance-build share: kernel traces of the C3 / C4 shapes (k_css_pack
# against the MDS kernel) and the GD_CSS_PROFILE phase cycles of the same shapes from the
# tools/ab/cssprof variant (build it first: tools/build_variant.sh cssprof -DGD_CSS_PROFILE).
# usage: tools/profile_round.sh r04    (then: python tools/summarize_prof.py r04)
set -o pipefail
R=${1:-r04}
O=gpurun_out/$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
timeout -k 10 120 tools/ubench_valu > $O/ubench_valu.txt 2>&1 &&
timeout -k 10 120 tools/ubench_mfma64 > $O/ubench_mfma64.txt 2>&1 &&
timeout -k 10 420 python3 bench.py --c45-steps 1 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu --c45-steps 1 > $O/ktrace_bench.json 2> $O/ktrace.err &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-css --no-extra > $O/pmc_fetch.json 2> $O/pmc_fetch.err &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-css --no-extra > $O/pmc_write.json 2> $O/pmc_write.err &&
timeout -s KILL 200 rocprofv3 --pmc $SQ -d $O/pmc_valu -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-css --no-extra > $O/pmc_valu.json 2> $O/pmc_valu.err &&
timeout -s KILL 200 rocprofv3 --pmc $SQ -d $O/pmc_c3 -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --css-steps 1 --no-extra --no-c45 > $O/pmc_c3.json 2> $O/pmc_c3.err &&
POP=40 NCH=4 RUNS=0 STEPS=1 timeout -s KILL 200 rocprofv3 --pmc $SQ -d $O/pmc_c4 -o run --output-format csv -- \
    python3 tools/css_time.py > $O/pmc_c4.txt 2> $O/pmc_c4.err &&
POP=40 NCH=1 RUNS=1000 TRES=10 STEPS=1 timeout -s KILL 200 rocprofv3 --pmc $SQ -d $O/pmc_c5 -o run \
    --output-format csv -- python3 tools/css_time.py > $O/pmc_c5.txt 2> $O/pmc_c5.err &&
POP=40 NCH=1 RUNS=1000 TRES=10 STEPS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    GRBM_GUI_ACTIVE SQ_WAVES -d $O/pmc_c5_mfma -o run --output-format csv -- python3 tools/css_time.py \
    > $O/pmc_c5_mfma.txt 2> $O/pmc_c5_mfma.err &&
POP=20 NCH=4 RUNS=0 STEPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_c3 -o run --output-format csv -- \
    python3 tools/css_time.py > $O/kt_c3.txt 2> $O/kt_c3.err &&
POP=40 NCH=4 RUNS=0 STEPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_c4 -o run --output-format csv -- \
    python3 tools/css_time.py > $O/kt_c4.txt 2> $O/kt_c4.err &&
GDSCAN_LIB=tools/ab/cssprof/libgdscan.so POP=20 NCH=4 RUNS=0 STEPS=1 timeout -k 10 200 python3 tools/css_time.py \
    > $O/ph_c3.txt 2> $O/ph_c3.err &&
GDSCAN_LIB=tools/ab/cssprof/libgdscan.so POP=40 NCH=4 RUNS=0 STEPS=1 timeout -k 10 200 python3 tools/css_time.py \
    > $O/ph_c4.txt 2> $O/ph_c4.err
echo "profile_round exit $?"
