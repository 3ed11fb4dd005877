set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s16
GD_CSS_OVERLAP_STREAM=low timeout -k 10 600 python -u -m pytest tests/test_css_perm_isolated.py tests/test_css_gpu.py tests/test_css_chained.py tests/test_shard_gpu.py tests/test_compat_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s16/t.log 2>&1 ; \
c5() { POP=40 NCH=$1 RUNS=1000 TRES=10 STEPS=2 timeout -k 10 120 python tools/css_time.py >> gpurun_out/s16/$2.txt 2>&1; }
GD_CSS_OVERLAP_STREAM=off c5 1 off && GD_CSS_OVERLAP_STREAM=low c5 1 low4 && GD_CSS_OVERLAP_STREAM=high c5 1 high4 && \
GD_CSS_OVERLAP_STREAM=low GD_CSS_OVERLAP_GROUPS=2 c5 1 low2 && GD_CSS_OVERLAP_STREAM=low GD_CSS_OVERLAP_GROUPS=8 c5 1 low8 && \
GD_CSS_OVERLAP_STREAM=off c5 4 off_n4 && GD_CSS_OVERLAP_STREAM=low c5 4 low4_n4 && GD_CSS_OVERLAP_STREAM=high c5 4 high4_n4
echo "exit $?"
