set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s23
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/s23/t.log 2>&1 ; \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s23/smoke.log 2>&1 && \
timeout -k 10 420 python3 bench.py > gpurun_out/s23/bench.json 2> gpurun_out/s23/bench.err
echo "exit $?"
