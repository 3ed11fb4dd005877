# FET scheduled-scan sweep with the cycle-profile variant (varlib/wprof) beside the regular build
set -o pipefail
O=gpurun_out/${OUT:-s4}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
IFS=';' read -ra CFGS <<< "${CFGS:-GD_FET_X=0}"
for cfg in "${CFGS[@]}"; do
  env $cfg timeout -k 10 120 python bench.py --no-css --no-extra --no-cpu --steps 20 --warmup 3 > $O/b.json 2> $O/b.err || exit 1
  echo "$cfg $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['stage_ms'].items()})")"
  if [ -n "$WPROF" ]; then
  env GDSCAN_LIB=varlib/wprof/libgdscan.so $cfg timeout -k 10 120 python bench.py --no-css --no-extra --no-cpu --steps 16 --warmup 1 > $O/bp.json 2> $O/bp.err || exit 1
  grep fet-wprof $O/bp.err | tail -1
  fi
done
