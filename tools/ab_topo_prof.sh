#!/bin/bash
# GPU box: KPSIM_PROFILE segment cycles of the config-3 Solve with each library under tools/ab/ (KPSIM_LIB override)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in tools/ab/*.so; do
  n=$(basename $lib .so)
  KPSIM_PROFILE=1 KPSIM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-consolidation --no-launch --no-reserved --steps 1 --warmup 0 > gpurun_out/abp_$n.json 2> gpurun_out/abp_$n.err || { tail -5 gpurun_out/abp_$n.err; exit 1; }
  echo "== $n"; grep "solve loop segments" gpurun_out/abp_$n.err | tail -1
  python3 -c "
import json; b=json.load(open('gpurun_out/abp_$n.json')); t=b['topology']
print('ffd %.1f' % t['kernel_ms']['ffd'], {k: v for k, v in t['ffd_counters'].items() if v})"
done
