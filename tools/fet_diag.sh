set -o pipefail
bash tools/pmc_valu.sh fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd/lib/libgdscan.so v10/main &&
for v in nodraw norank nostage; do bash tools/pmc_valu.sh tools/variants/$v/libgdscan.so v10/$v || exit 1; done &&
GDSCAN_LIB=tools/variants/fetprof/libgdscan.so timeout -k 10 100 python bench.py --no-cpu --no-css --no-extra --steps 8 > gpurun_out/v10/prof.json 2> gpurun_out/v10/prof.err
