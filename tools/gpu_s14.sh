set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s14
for v in fb8 fb4; do
  for g in 1 2; do
    GDSCAN_LIB=tools/variants/$v/libgdscan.so GD_GROUPS=$g timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/s14/${v}_g$g.json 2> gpurun_out/s14/${v}_g$g.err || exit 1
  done
done
GD_GROUPS=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-css --no-extra --no-cpu > gpurun_out/s14/fb16_g1.json 2> gpurun_out/s14/fb16_g1.err
echo "exit $?"
