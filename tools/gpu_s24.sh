set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s24
timeout -k 10 600 python -u -m pytest tests/test_fet_gpu.py tests/test_fet_exact.py tests/test_shard_gpu.py tests/test_compat_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s24/t.log 2>&1 && \
run() { timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/s24/$1.json 2> gpurun_out/s24/$1.err; }
run new && GDSCAN_LIB=tools/variants/kbold/libgdscan.so run old && GDSCAN_LIB=tools/variants/kbmag/libgdscan.so run mag && \
run new2 && GDSCAN_LIB=tools/variants/kbold/libgdscan.so run old2 && GDSCAN_LIB=tools/variants/kbmag/libgdscan.so run mag2
echo "exit $?"
