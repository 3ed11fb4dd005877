#!/bin/bash
# One GPU-box profiling pass (per round), each measurement in a run of its own:
#   the VALU / FP64-MFMA microbenchmarks (issue rate per op class);
#   the default bench line (python3 bench.py, as the driver runs it) and a two-rank rehearsal
#     (--gpus 2, both ranks on the one GPU over gloo) that carries cpu_baseline at N = 2;
#   kernel traces + stats PER LEG: the FET bench (C2) -- also the source of the one-scan
#     timeline --, and tools/css_time.py at the C3, C4 and C5 shapes;
#   PMC passes: FETCH_SIZE and WRITE_SIZE (HBM traffic) and the SQ issue counters (+
#     GRBM_GUI_ACTIVE, the kernel's clock cycles) of the FET scan kernels, the C3
#     (k_css_pack + k_css_mds_h40), C4 (k_css_mds_t80) and C5 permutation (k_css_perm<80>)
#     kernels, and the C5 matrix-core busy cycles;
#   phase cycles of the GD_CSS_PROFILE (varlib/cssprof) and GD_PERM_PROFILE (varlib/pprof)
#     builds at the C3 / C4 / C5 shapes.  Build the two variants first:
#       SRC="gd_css_t80 gd_css_h40" tools/build_variant.sh cssprof -DGD_CSS_PROFILE
#       SRC=gd_css_perm tools/build_variant.sh pprof -DGD_PERM_PROFILE
# Every GPU step has its own time limit; the steps are chained with &&.
# usage: tools/profile_round.sh r05    (then: python tools/summarize_prof.py r05)
set -o pipefail
R=${1:-r05}
O=gpurun_out/$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
C3="POP=20 NCH=20 RUNS=0"
C4="POP=40 NCH=4 RUNS=0"
C5="POP=40 NCH=1 RUNS=1000 TRES=10"
echo "profile_round $R: microbenchmarks" &&
timeout -k 10 120 tools/ubench_valu > $O/ubench_valu.txt 2>&1 &&
timeout -k 10 120 tools/ubench_mfma64 > $O/ubench_mfma64.txt 2>&1 &&
echo "bench (default)" &&
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err &&
echo "bench --gpus 2 (two ranks on the one GPU)" &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --no-extra --no-css --cpu-chroms 4 \
    > $O/bench_g2.json 2> $O/bench_g2.err &&
echo "kernel traces per leg" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_fet -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu --no-css --no-extra > $O/kt_fet.json 2> $O/kt_fet.err &&
env $C3 STEPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_c3 -o run --output-format csv -- \
    python3 tools/css_time.py > $O/kt_c3.txt 2> $O/kt_c3.err &&
env $C4 STEPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_c4 -o run --output-format csv -- \
    python3 tools/css_time.py > $O/kt_c4.txt 2> $O/kt_c4.err &&
env $C5 STEPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o run --output-format csv -- \
    python3 tools/css_time.py > $O/kt_c5.txt 2> $O/kt_c5.err &&
echo "PMC passes" &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-css --no-extra > $O/pmc_fetch.json 2> $O/pmc_fetch.err &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-css --no-extra > $O/pmc_write.json 2> $O/pmc_write.err &&
timeout -s KILL 200 rocprofv3 --pmc $SQ -d $O/pmc_valu -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-css --no-extra > $O/pmc_valu.json 2> $O/pmc_valu.err &&
env $C3 STEPS=1 timeout -s KILL 200 rocprofv3 --pmc $SQ -d $O/pmc_c3 -o run --output-format csv -- \
    python3 tools/css_time.py > $O/pmc_c3.txt 2> $O/pmc_c3.err &&
env $C4 STEPS=1 timeout -s KILL 200 rocprofv3 --pmc $SQ -d $O/pmc_c4 -o run --output-format csv -- \
    python3 tools/css_time.py > $O/pmc_c4.txt 2> $O/pmc_c4.err &&
env $C5 STEPS=1 timeout -s KILL 200 rocprofv3 --pmc $SQ -d $O/pmc_c5 -o run --output-format csv -- \
    python3 tools/css_time.py > $O/pmc_c5.txt 2> $O/pmc_c5.err &&
env $C5 STEPS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \
    -d $O/pmc_c5_mfma -o run --output-format csv -- python3 tools/css_time.py > $O/pmc_c5_mfma.txt 2> $O/pmc_c5_mfma.err &&
echo "phase profiles" &&
env $C3 STEPS=1 GDSCAN_LIB=varlib/cssprof/libgdscan.so timeout -k 10 200 python3 tools/css_time.py \
    > $O/ph_c3.txt 2> $O/ph_c3.err &&
env $C4 STEPS=1 GDSCAN_LIB=varlib/cssprof/libgdscan.so timeout -k 10 200 python3 tools/css_time.py \
    > $O/ph_c4.txt 2> $O/ph_c4.err &&
env $C5 STEPS=1 GDSCAN_LIB=varlib/pprof/libgdscan.so timeout -k 10 200 python3 tools/css_time.py \
    > $O/ph_c5.txt 2> $O/ph_c5.err
echo "profile_round exit $?"
