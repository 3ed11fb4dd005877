set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s9
timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py tests/test_css_gpu.py tests/test_css_big.py tests/test_css_options.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s9/t.log 2>&1 ; \
bash tools/ab_perm.sh s9 sc4 sc5 sc5prof sc4 sc5 && \
GDSCAN_LIB=tools/variants/csprof/libgdscan.so POP=40 NCH=4 STEPS=2 timeout -k 10 120 python tools/css_time.py > gpurun_out/s9/csprof40.txt 2>&1 && \
GDSCAN_LIB=tools/variants/csprof/libgdscan.so POP=20 NCH=4 STEPS=2 timeout -k 10 120 python tools/css_time.py > gpurun_out/s9/csprof20.txt 2>&1
echo "exit $?"
