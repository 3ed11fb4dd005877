set -o pipefail
O=gpurun_out/${OUT:-s10}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_fet_gpu.py tests/test_compat_gpu.py tests/test_packed.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
IFS=';' read -ra CFGS <<< "${CFGS:-GD_FET_X=0}"
for cfg in "${CFGS[@]}"; do
  env $cfg timeout -k 10 120 python bench.py --no-css --no-extra --no-cpu --steps 20 --warmup 3 > $O/b.json 2> $O/b.err || exit 1
  echo "$cfg $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['stage_ms'].items()})")"
done
if [ -n "$KT" ]; then
env $KTENV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --no-css --no-extra --no-cpu --steps 5 --warmup 1 > $O/kt.json 2> $O/kt.err
fi
echo done
