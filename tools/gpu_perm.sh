# C5 permutation A/B on the GPU box: the isolated permutation tests, then tools/css_time.py at
# the C5 shape (1 x 500k SNPs, 40+40, treshold 10, 1000 runs) per library (LIBS: ';'-separated
# GDSCAN_LIB paths; "" = the regular build); PROF=<lib>: its perm-prof phase line; PMC=1: the
# permutation kernel's counters (one rocprofv3 pass per group)
set -o pipefail
O=gpurun_out/${OUT:-perm}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
REG=fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd/lib/libgdscan.so
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_css_perm_isolated.py} -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
IFS=';' read -ra LIBS <<< "${LIBS:-}"
for lib in "" "${LIBS[@]}"; do
  GDSCAN_LIB=${lib:-$REG} POP=40 NCH=1 RUNS=1000 TRES=10 STEPS=${STEPS:-3} \
    timeout -k 10 200 python tools/css_time.py > $O/t.log 2>&1 || { echo "css_time failed ($lib)"; tail -20 $O/t.log; exit 1; }
  echo "${lib:-regular}: $(grep '^CSS' $O/t.log)"
done
if [ -n "$PROF" ]; then
  GDSCAN_LIB=$PROF POP=40 NCH=1 RUNS=1000 TRES=10 STEPS=1 timeout -k 10 200 python tools/css_time.py > $O/p.log 2>&1 || exit 1
  grep -E "perm-prof" $O/p.log | tail -1
fi
if [ -n "$PMC" ]; then
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"; do
    i=$((i+1))
    POP=40 NCH=1 RUNS=1000 TRES=10 STEPS=1 timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/pmc$i -o run --output-format csv -- python tools/css_time.py > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
  done
  for i in 1 2; do for f in $(find $O/pmc$i -name '*counter_collection.csv'); do python tools/pmc_sum.py $f perm; done; done
fi
echo done
