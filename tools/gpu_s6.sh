set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s6
GDSCAN_LIB=tools/variants/sc3c2/libgdscan.so timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py tests/test_css_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s6/t.log 2>&1 ; \
bash tools/ab_perm.sh s6 sc3 sc3c2 sc3c2prof sc3 sc3c2
echo "exit $?"
