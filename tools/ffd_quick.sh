#!/bin/bash
# GPU-box check of an ffd-kernel / eval change: Solve, topology, preference, reservation and consolidation parity
# suites, then the config2 and config3 Solve legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_topology.py tests/test_gpu_preferences.py tests/test_gpu_consolidation.py tests/test_gpu_reserved.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tf.log 2>&1 || { tail -30 gpurun_out/tf.log; exit 1; }
tail -2 gpurun_out/tf.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-consolidation --no-launch --no-reserved ${BENCH_EXTRA:-} --steps 5 --warmup 1 > gpurun_out/bfq.json 2> gpurun_out/bfq.err || { tail -5 gpurun_out/bfq.err; exit 1; }
python3 -c "
import json; b=json.load(open('gpurun_out/bfq.json')); t=b.get('topology') or {}
print('pods/s %.0f ms %.3f ffd %.3f' % (b['value'], b['ms_per_step'], b['kernel_ms']['ffd']), 'topo ffd', (t.get('kernel_ms') or {}).get('ffd'))"
