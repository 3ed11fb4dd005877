#!/bin/bash
# End-of-round GPU pass: the GPU test suite, smoke(), then tools/profile_round.sh $1.
set -o pipefail
R=${1:-r02}
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/$R/gputest.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 &&
bash tools/profile_round.sh $R
