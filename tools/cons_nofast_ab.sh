#!/bin/bash
# GPU box: consolidation legs (config 4, config 4 replace) with and without the fast probe variant (KPSIM_CONS_NOFAST=1:
# every probe on the FULL variant), to see what the fast-then-FULL hand-over costs the replace pass's critical path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 1; do
  KPSIM_CONS_NOFAST=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-topology --no-reserved --no-launch --steps 3 --warmup 1 > gpurun_out/nf_$v.json 2> gpurun_out/nf_$v.err || { tail -5 gpurun_out/nf_$v.err; exit 1; }
  python3 -c "
import json; b=json.load(open('gpurun_out/nf_$v.json'))
print('NOFAST=$v', 'config4', b['consolidation']['kernel_ms_rank0'], 'replace', b['consolidation_replace']['kernel_ms_rank0'], 'stages', b.get('stage_cycles_per_pod'))"
done
