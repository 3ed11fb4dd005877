set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s3
timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py tests/test_css_gpu.py tests/test_css_chained.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3/t.log 2>&1 && \
bash tools/ab_perm.sh s3 base fy2 fy2prof base fy2
echo "exit $?"
