set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s21
timeout -k 10 900 python -u -m pytest tests/test_fet_gpu.py tests/test_fet_exact.py tests/test_stats.py tests/test_compat_gpu.py tests/test_tools_gpu.py tests/test_regions.py tests/test_css_gpu.py tests/test_css_big.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s21/t.log 2>&1 ; \
run() { timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/s21/$1.json 2> gpurun_out/s21/$1.err; }
GD_GROUPS=1 run new_g1 && GD_GROUPS=2 run new_g2 && \
GDSCAN_LIB=tools/variants/oldkb/libgdscan.so GD_GROUPS=1 run old_g1 && GDSCAN_LIB=tools/variants/oldkb/libgdscan.so GD_GROUPS=2 run old_g2 && \
GD_GROUPS=1 run new_g1b && GDSCAN_LIB=tools/variants/oldkb/libgdscan.so GD_GROUPS=1 run old_g1b
echo "exit $?"
