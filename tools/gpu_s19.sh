set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s19
GDSCAN_LIB=tools/variants/mlds/libgdscan.so timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s19/t.log 2>&1 ; \
bash tools/ab_perm.sh s19 base mlds base mlds
echo "exit $?"
