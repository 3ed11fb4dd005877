# Per-phase counters of the permutation kernel (C5 shape, k_css_perm<80>): builds run every
# window's full mcR permutations (PERM_DIAG_NOEXIT) and skip phases (PERM_DIAG_SKIP bits:
# 1 draws, 2 compositions, 4 scores); differences of their SQ counters per dispatch give each
# phase's share.  Build first (CPU):
#   for v in "all:0" "nos:4" "noc:6" "nod:7"; do n=${v%%:*}; k=${v##*:};
#     SRC=gd_css_perm tools/build_variant.sh pp_$n "-DPERM_DIAG_NOEXIT=1 -DPERM_DIAG_SKIP=$k"; done
set -o pipefail
O=gpurun_out/${OUT:-pphase}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
for n in all nos noc nod; do
  GDSCAN_LIB=varlib/pp_$n/libgdscan.so POP=40 NCH=1 RUNS=1000 TRES=10 STEPS=1 timeout -s KILL 150 rocprofv3 --pmc $SQ \
      -d $O/pmc_$n -o run --output-format csv -- python3 tools/css_time.py > $O/pmc_$n.txt 2> $O/pmc_$n.err || { echo "pass $n failed"; exit 1; }
  echo "$n $(grep '^CSS' $O/pmc_$n.txt)"
done
echo done
