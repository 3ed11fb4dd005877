set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s25
run() { timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/s25/$1.json 2> gpurun_out/s25/$1.err; }
run new && GD_GROUPS=2 run g2 && GDSCAN_LIB=tools/variants/kbch8/libgdscan.so run ch8 && GDSCAN_LIB=tools/variants/kbch2/libgdscan.so run ch2 && \
run new2 && GD_GROUPS=2 run g2b && GDSCAN_LIB=tools/variants/kbch8/libgdscan.so run ch8b && GDSCAN_LIB=tools/variants/kbch2/libgdscan.so run ch2b && \
GDSCAN_LIB=tools/variants/fetprof/libgdscan.so run prof
echo "exit $?"
