# CSS MDS A/B on the GPU box: parity tests, then tools/css_time.py per library (LIBS: ';'-separated
# GDSCAN_LIB paths, "" = the regular build) at the C3 and C4 shapes
set -o pipefail
O=gpurun_out/${OUT:-css}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_css_gpu.py} -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
IFS=';' read -ra LIBS <<< "${LIBS:-}"
for lib in "" "${LIBS[@]}"; do
  for pop in ${POPS:-20 40}; do
    nch=20; [ $pop = 40 ] && nch=4
    GDSCAN_LIB=${lib:-fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd/lib/libgdscan.so} POP=$pop NCH=$nch STEPS=${STEPS:-5} \
      timeout -k 10 200 python tools/css_time.py > $O/t.log 2>&1 || { echo "css_time failed ($lib $pop)"; tail -20 $O/t.log; exit 1; }
    echo "${lib:-regular} pop=$pop: $(grep '^CSS' $O/t.log)"
  done
done
echo done
