set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s15
timeout -k 10 600 python -u -m pytest tests/test_fet_gpu.py tests/test_fet_exact.py tests/test_stats.py tests/test_compat_gpu.py tests/test_tools_gpu.py tests/test_packed.py tests/test_regions.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s15/t.log 2>&1 ; \
run() { timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/s15/$1.json 2> gpurun_out/s15/$1.err; }
GD_GROUPS=1 run fb16_g1 && GD_GROUPS=2 run fb16_g2 && \
GDSCAN_LIB=tools/variants/fb8/libgdscan.so GD_GROUPS=1 run fb8_g1 && GDSCAN_LIB=tools/variants/fb8/libgdscan.so GD_GROUPS=2 run fb8_g2 && \
GDSCAN_LIB=tools/variants/fb4/libgdscan.so GD_GROUPS=1 run fb4_g1 && \
GD_FET_KBOUNDS=1 GD_GROUPS=2 run kb_g2 && GD_FET_KBOUNDS=1 GD_GROUPS=1 run kb_g1
echo "exit $?"
