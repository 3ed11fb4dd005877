set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof80
GDSCAN_LIB=tools/variants/prof/libgdscan.so POP=40 NCH=4 STEPS=2 timeout -k 10 120 python tools/css_time.py > gpurun_out/prof80/out.txt 2>&1
