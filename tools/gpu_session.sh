#!/bin/bash
# One parameterised GPU-box session (replaces the one-off gpu_s*.sh scripts of round 3).
# Every step runs under its own time limit; the first failing step ends the session.
#
# usage: tools/gpu_session.sh OUT STEP [STEP ...]      (outputs under gpurun_out/OUT/)
#   tests[=FILES]        pytest -m gpu over tests/ (or the listed test files, comma separated)
#   testlib=TAG          the FET/compat GPU tests against tools/ab/TAG/libgdscan.so
#   smoke                __graft_entry__.smoke()
#   bench[=ARGS]         python bench.py ARGS (underscores in ARGS become spaces)
#   fet[=TAG]            FET-only bench (20 steps), libgdscan.so of tools/ab/TAG if given
#   fetenv=K=V,...       FET-only bench with environment variables set (e.g. GD_GROUPS=2)
#   valu[=TAG]           SQ VALU/LDS counters of the FET-only bench, variant TAG if given
#   css[=ENV]            tools/css_time.py with ENV (e.g. POP=40,NCH=4,RUNS=0,STEPS=5)
# Variants are built on the CPU beforehand: tools/build_variant.sh TAG "-DFLAG ..."
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
lib() { if [ -n "$1" ]; then echo "tools/ab/$1/libgdscan.so"; else echo ""; fi; }
i=0
for S in "$@"; do
  i=$((i + 1)); K=${S%%=*}; V=""; [ "$K" != "$S" ] && V=${S#*=}
  case $K in
    tests)
      F=tests; [ -n "$V" ] && F=${V//,/ }
      timeout -k 10 900 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread \
        > $O/$i.tests.log 2>&1 ;;
    testlib)
      GDSCAN_LIB=$(lib "$V") timeout -k 10 600 python -u -m pytest tests/test_fet_gpu.py tests/test_compat_gpu.py \
        tests/test_packed.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/$i.testlib$V.log 2>&1 ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/$i.smoke.log 2>&1 ;;
    bench)
      timeout -k 10 600 python3 bench.py ${V//_/ } > $O/$i.bench.json 2> $O/$i.bench.err ;;
    fet)
      L=$(lib "$V"); env ${L:+GDSCAN_LIB=$L} timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra \
        --no-cpu > $O/$i.fet$V.json 2> $O/$i.fet$V.err ;;
    fetenv)
      env ${V//,/ } timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra \
        --no-cpu > $O/$i.fetenv.json 2> $O/$i.fetenv.err ;;
    valu)
      L=$(lib "$V"); env ${L:+GDSCAN_LIB=$L} timeout -s KILL 150 rocprofv3 --pmc $SQ -d $O/$i.valu$V -o run \
        --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-css --no-extra \
        > $O/$i.valu$V.json 2> $O/$i.valu$V.err ;;
    css)
      env ${V//,/ } timeout -k 10 300 python3 tools/css_time.py > $O/$i.css.txt 2> $O/$i.css.err ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
  rc=$?
  echo "step $i $S rc $rc" | tee -a $O/steps.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
