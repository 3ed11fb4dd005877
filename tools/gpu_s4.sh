set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s4
timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py tests/test_css_gpu.py tests/test_css_chained.py tests/test_packed.py tests/test_css_options.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s4/t.log 2>&1 ; \
bash tools/ab_perm.sh s4 base sc1 sc2 sc2prof base sc2
echo "exit $?"
