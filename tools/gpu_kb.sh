# k_bounds variants: per-variant bench (default groups) and the bounds kernel's average time (kernel trace, one group)
set -o pipefail
O=gpurun_out/${OUT:-kb}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in base kb8 kbpf kbpf8 kb2pf; do
  L=""; [ "$v" != base ] && L="GDSCAN_LIB=varlib/$v/libgdscan.so"
  env $L timeout -k 10 120 python bench.py --no-css --no-extra --no-cpu --steps 20 --warmup 3 > $O/b.json 2> $O/b.err || exit 1
  ms=$(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['ms_per_step'],4), round(d['stage_ms']['scan'],4))")
  env $L GD_GROUPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o run --output-format csv -- python bench.py --no-css --no-extra --no-cpu --steps 5 --warmup 1 > /dev/null 2> $O/kt.err || exit 1
  kb=$(python -c "
import csv
r=[x for x in csv.DictReader(open('$O/kt_$v/run_kernel_stats.csv')) if x['Name'].startswith('k_bounds')]
print(r[0]['AverageNs'] if r else 'na')")
  echo "$v step/scan $ms k_bounds_avg_ns $kb"
done
