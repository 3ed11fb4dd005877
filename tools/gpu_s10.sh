set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s10
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py tests/test_css_perm_isolated.py tests/test_css_gpu.py tests/test_packed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s10/t.log 2>&1 ; \
bash tools/ab_perm.sh s10 sc5 sc6 sc6prof sc5 sc6
echo "exit $?"
