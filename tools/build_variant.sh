#!/bin/bash
# Build an A/B variant of libgdscan.so: csrc/gd_css_t80.hip (or $SRC) recompiled with
# extra flags, linked with the other objects of the regular build.
# usage: tools/build_variant.sh NAME "-DGD_CSS_PROFILE ..."   -> varlib/NAME/libgdscan.so (git-ignored; delete after the A/B session: it travels with every gpurun call)
set -e
NAME=$1; FLAGS=$2; SRC=${SRC:-gd_css_t80}
P=$(cd "$(dirname "$0")/.." && pwd)/fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd
OUT=$(cd "$(dirname "$0")/.." && pwd)/varlib/$NAME
mkdir -p "$OUT"
make -s -C "$P" >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w $FLAGS \
    -c "$P/csrc/$SRC.hip" -o "$OUT/$SRC.o"
OBJS=$(ls "$P"/build/*.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libgdscan.so" $OBJS "$OUT/$SRC.o" -lpthread
echo "$OUT/libgdscan.so"
