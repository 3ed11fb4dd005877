set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s26
timeout -k 10 600 python -u -m pytest tests/test_fet_gpu.py tests/test_shard_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s26/t.log 2>&1 || exit 1
run() { timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/s26/$1.json 2> gpurun_out/s26/$1.err; }
V() { GDSCAN_LIB=tools/variants/$1/libgdscan.so run $1$2; }
for r in a b; do run new$r && V stu8 $r && V stu12 $r && V stu16 $r && V spn640 $r && V spn640u8 $r && V spn640u12 $r || exit 1; done
echo "exit $?"
