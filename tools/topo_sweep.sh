#!/bin/bash
# GPU box: config-3 (topology) Solve time per KPSIM_TOPO_CANDS value, then the topology parity suite at the value given
# as $1.  Usage: bash tools/topo_sweep.sh <cands for the parity run> [values to time...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PV=${1:-2}; shift
for v in "${@:-1 2 4 8}"; do
  KPSIM_TOPO_CANDS=$v timeout -k 10 200 python bench.py --no-consolidation --no-launch --no-reserved --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/ts_$v.json 2> gpurun_out/ts_$v.err || { tail -3 gpurun_out/ts_$v.err; exit 1; }
  python3 -c "import json; t=json.load(open('gpurun_out/ts_$v.json'))['topology']; print('cands $v: ffd_topo %.1f ms' % t['kernel_ms']['ffd'], t['solve_stats'])"
done
KPSIM_TOPO_CANDS=$PV timeout -k 10 500 python -u -m pytest tests/test_gpu_topology.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tt.log 2>&1 || { tail -20 gpurun_out/tt.log; exit 1; }
tail -1 gpurun_out/tt.log
