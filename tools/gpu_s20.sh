set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s20
timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py tests/test_css_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s20/t.log 2>&1 ; \
GDSCAN_LIB=tools/variants/mlds/libgdscan.so timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s20/t_mlds.log 2>&1 ; \
bash tools/ab_perm.sh s20 base mlds base mlds
echo "exit $?"
