#!/bin/bash
# Build an A/B variant of libgdscan.so: csrc/gd_css_t80.hip (or the sources named in $SRC,
# space-separated, without .hip) recompiled with extra flags, linked with the other objects of
# the regular build.
# usage: [SRC="gd_css_t80 gd_css_h40"] tools/build_variant.sh NAME "-DGD_CSS_PROFILE ..."
#   -> varlib/NAME/libgdscan.so (git-ignored; delete after the A/B session: it travels with every gpurun call)
set -e
NAME=$1; FLAGS=$2; SRC=${SRC:-gd_css_t80}
P=$(cd "$(dirname "$0")/.." && pwd)/fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd
OUT=$(cd "$(dirname "$0")/.." && pwd)/varlib/$NAME
mkdir -p "$OUT"
make -s -C "$P" >/dev/null
OBJS=$(ls "$P"/build/*.o)
pids=()
for s in $SRC; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w $FLAGS \
      -c "$P/csrc/$s.hip" -o "$OUT/$s.o" &
  pids+=($!)
  OBJS=$(echo "$OBJS" | grep -v "/$s.o$")
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libgdscan.so" $OBJS $(for s in $SRC; do echo "$OUT/$s.o"; done) -lpthread
echo "$OUT/libgdscan.so"
