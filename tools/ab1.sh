set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab1
GDSCAN_LIB=tools/variants/pipe/libgdscan.so timeout -k 10 300 python -u -m pytest tests/test_css_gpu.py tests/test_css_perm_isolated.py -x -q -k "40-40 or 33-40 or 45-45 or 30-42 or 43-30 or largest or 64-64" --timeout 120 --timeout-method thread > gpurun_out/ab1/test.log 2>&1 || exit 1
POPS="40" bash tools/ab_css.sh ab1 f4 pipe f4 pipe
