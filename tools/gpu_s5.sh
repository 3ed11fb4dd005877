set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s5
timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py tests/test_css_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s5/t.log 2>&1 ; \
bash tools/ab_perm.sh s5 base sc2 sc3 sc3p sc3n4 sc3prof sc3pprof sc3 sc3p
echo "exit $?"
