#!/bin/bash
# GPU box: the config-5 (reserved) Solve leg with each library under tools/ab/ (KPSIM_LIB override)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in tools/ab/*.so; do
  n=$(basename $lib .so)
  KPSIM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-consolidation --no-launch --no-topology --steps 2 --warmup 1 > gpurun_out/abr_$n.json 2> gpurun_out/abr_$n.err || { tail -5 gpurun_out/abr_$n.err; exit 1; }
  python3 -c "
import json; b=json.load(open('gpurun_out/abr_$n.json'))
print('$n config2 ffd %.2f config5 ffd %.1f' % (b['kernel_ms']['ffd'], b['reserved']['kernel_ms']['ffd']))"
done
