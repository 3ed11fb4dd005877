set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s18
timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py tests/test_css_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/s18/t.log 2>&1
echo "exit $?"
