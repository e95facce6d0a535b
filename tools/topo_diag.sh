#!/bin/bash
# GPU box: config-3 stage split (libkpsim_diag.so, KP_DIAG_SPLIT): offerings+totals / sweep / join+min, team and no-team
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in team noteam; do
  [ $v = noteam ] && continue
  KPSIM_LIB=$PWD/karpenter-provider-aws_amd/lib/libkpsim_diag.so KPSIM_PROFILE=1 timeout -k 10 200 python bench.py --no-consolidation --no-launch --no-reserved --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/td_$v.json 2> gpurun_out/td_$v.err || { tail -3 gpurun_out/td_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/td_$v.json'))['topology']; c=d['ffd_counters']
print('$v', d['kernel_ms']['ffd'], {k: c[k] for k in ('cyc_slow_eval','ev_req','ev_mask','ev_off','ev_types','ev_min','ev_calls','rej_requirements','rej_topology','rej_types','rej_min_values','cyc_topo_setup','cyc_topo_scan','cyc_templates')})"
done
