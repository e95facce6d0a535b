#!/bin/bash
# GPU box: the config-5 (reserved) Solve leg under each diagnostics switch of the FFD kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base KPSIM_NO_TEAM_FIRST KPSIM_NO_NOOP KPSIM_NO_BLOCK_SORT; do
  ( [ $v != base ] && export $v=1; timeout -k 10 200 python bench.py --no-cpu-baseline --no-consolidation --no-launch --no-topology --steps 2 --warmup 1 > gpurun_out/ra_$v.json 2> gpurun_out/ra_$v.err ) || { tail -3 gpurun_out/ra_$v.err; exit 1; }
  python3 -c "
import json; b=json.load(open('gpurun_out/ra_$v.json')); r=b['reserved']
print('$v', 'config2 ffd %.2f' % b['kernel_ms']['ffd'], 'config5 ffd %.1f' % r['kernel_ms']['ffd'])"
done
