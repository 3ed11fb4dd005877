# FET bench A/B on the GPU box: the FET GPU tests on the regular build, then bench.py's FET line
# alternated between varlib/old and the regular build (3 rounds, 40 steps each)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abf
timeout -k 10 400 python -u -m pytest tests/test_fet_gpu.py tests/test_compat_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abf/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/abf/tests.log; exit 1; }
tail -1 gpurun_out/abf/tests.log
NEW=fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd/lib/libgdscan.so
for i in 1 2 3; do
  for lib in varlib/old/libgdscan.so $NEW; do
    GDSCAN_LIB=$lib timeout -k 10 120 python3 bench.py --steps 40 --warmup 3 --no-cpu --no-css --no-extra > gpurun_out/abf/o.json 2> gpurun_out/abf/e.log || { echo FAIL $lib; tail -5 gpurun_out/abf/e.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/abf/o.json').read().strip().splitlines()[-1]);print('$lib'[:12], round(d['ms_per_step'],4), round(d['stage_ms']['scan'],4))"
  done
done
