set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s7
timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py tests/test_css_gpu.py tests/test_css_big.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s7/t.log 2>&1 ; \
bash tools/ab_perm.sh s7 sc3 sc4 sc4prof sc3 sc4 && \
bash tools/fet_groups.sh s7fet fetnodraw
echo "exit $?"
