# host-path (drop-in call) tests and bench legs on the GPU box
set -o pipefail
O=gpurun_out/${OUT:-h1}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_host_pack_gpu.py tests/test_compat_gpu.py tests/test_stats.py tests/test_tools_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --no-css --steps 10 > $O/b.json 2> $O/b.err || { echo BENCH FAILED; tail -20 $O/b.err; exit 1; }
python - <<'PY'
import json,os
d=json.load(open(os.environ.get('O','gpurun_out/h1')+'/b.json'))
print(d['ms_per_step'], json.dumps(d['host_path'])[:900])
print(json.dumps(d['c1'])[:1500])
print(json.dumps(d['cpu_baseline'])[:400])
PY
