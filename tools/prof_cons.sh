#!/bin/bash
# GPU box: the consolidation legs (config 4 delete, config4-replace) under KPSIM_PROFILE=1: the probes that bound each pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
KPSIM_PROFILE=1 timeout -k 10 300 python bench.py --no-launch --no-reserved --no-topology --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/pc.json 2> gpurun_out/pc.err || { tail -3 gpurun_out/pc.err; exit 1; }
grep "probes [0-9]*: longest\|slow-path pods" gpurun_out/pc.err || true
timeout -k 10 300 python bench.py --no-launch --no-reserved --no-topology --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/pcq.json 2> gpurun_out/pcq.err || { tail -3 gpurun_out/pcq.err; exit 1; }
python3 -c "
import json; q=json.load(open('gpurun_out/pcq.json'))
print('solve ms', q['ms_per_step'], 'ffd', q['kernel_ms']['ffd'])
for leg in ('consolidation', 'consolidation_replace'):
    c = q.get(leg) or {}
    print(leg, c.get('ms_per_step'), c.get('kernel_ms_rank0'))"
