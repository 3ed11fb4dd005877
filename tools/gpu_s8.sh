set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s8/t.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s8/smoke.log 2>&1 && \
bash tools/profile_r03.sh r03
echo "exit $?"
