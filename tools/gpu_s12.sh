set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s12
timeout -k 10 900 python -u -m pytest tests/test_fet_gpu.py tests/test_fet_exact.py tests/test_stats.py tests/test_compat_gpu.py tests/test_tools_gpu.py tests/test_packed.py tests/test_regions.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s12/t.log 2>&1 ; \
for g in 1 2 4; do GD_GROUPS=$g timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/s12/fb_g$g.json 2> gpurun_out/s12/fb_g$g.err || exit 1; done && \
GD_FET_KBOUNDS=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/s12/kb_g2.json 2> gpurun_out/s12/kb_g2.err
echo "exit $?"
