# FET scheduled-scan A/B on the GPU box (diagnostic knobs: GD_FET_* in csrc/gd_api.hip)
set -o pipefail
O=gpurun_out/${OUT:-s1}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [ -z "$NOTEST" ]; then
timeout -k 10 300 python -u -m pytest tests/test_fet_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
IFS=';' read -ra CFGS <<< "${CFGS:-}"
for cfg in "${CFGS[@]}"; do
  env $cfg timeout -k 10 120 python bench.py --no-css --no-extra --no-cpu --steps 20 --warmup 3 > $O/b.json 2> $O/b.err || exit 1
  python -c "import json,sys;d=json.load(open('$O/b.json'));print('$cfg', round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['stage_ms'].items()})"
done
if [ -n "$KT" ]; then
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --no-css --no-extra --no-cpu --steps 5 --warmup 1 > $O/kt.json 2> $O/kt.err
fi
echo done
