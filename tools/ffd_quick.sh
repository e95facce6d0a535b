#!/bin/bash
# GPU-box check of an ffd-kernel change: Solve parity suites, then the config2 Solve leg (10 steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_topology.py tests/test_gpu_preferences.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tf.log 2>&1 || { tail -30 gpurun_out/tf.log; exit 1; }
tail -2 gpurun_out/tf.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-consolidation --no-launch --no-topology --no-reserved --steps 10 --warmup 2 > gpurun_out/bfq.json 2> gpurun_out/bfq.err || { tail -5 gpurun_out/bfq.err; exit 1; }
python3 -c "
import json; b=json.load(open('gpurun_out/bfq.json')); print('pods/s %.0f ms %.3f ffd %.3f' % (b['value'], b['ms_per_step'], b['kernel_ms']['ffd']), b['solve_call_warm'])"
