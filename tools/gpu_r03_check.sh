set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t3.log 2>&1 && \
NCH=1 NSNP=100000 POP=80 STEPS=2 timeout -k 10 120 python tools/css_time.py > gpurun_out/big.log 2>&1 && \
NCH=1 NSNP=100000 POP=150 STEPS=2 timeout -k 10 120 python tools/css_time.py >> gpurun_out/big.log 2>&1 && \
NCH=1 NSNP=50000 POP=80 RUNS=1000 STEPS=1 timeout -k 10 200 python tools/css_time.py >> gpurun_out/big.log 2>&1
