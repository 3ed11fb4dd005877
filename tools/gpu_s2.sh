set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s2
bash tools/ab_perm.sh s2 base prof && \
timeout -k 10 600 python3 bench.py --gpus 2 --no-cpu > gpurun_out/s2/bench2.json 2> gpurun_out/s2/bench2.err
echo "exit $?"
