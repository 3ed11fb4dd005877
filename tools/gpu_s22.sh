set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s22
GDSCAN_LIB=tools/variants/kb8/libgdscan.so timeout -k 10 600 python -u -m pytest tests/test_fet_gpu.py tests/test_css_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s22/t.log 2>&1 ; \
run() { GDSCAN_LIB=tools/variants/$1/libgdscan.so timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/s22/$2.json 2> gpurun_out/s22/$2.err; }
run kb4 kb4a && run kb8 kb8a && run kb4 kb4b && run kb8 kb8b
echo "exit $?"
