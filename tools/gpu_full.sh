# full GPU suite + default bench line (round-end shape), each step under its own limit
set -o pipefail
O=gpurun_out/${OUT:-full}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
if [ -z "$NOBENCH" ]; then
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'], d['stage_ms'], {k:(v['value'] if isinstance(v,dict) and 'value' in v else None) for k,v in d.get('css',{}).items()})"
fi
