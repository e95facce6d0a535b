#!/bin/bash
# GPU-box A/B of kp_launch_select's host/device pipeline: launch parity tests, then the launch leg of bench.py per
# (sub-batches KPSIM_LAUNCH_SUB, worker spin KPSIM_POOL_SPIN_US) setting — kernel time, call time and host phases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_launch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lt.log 2>&1 || { tail -30 gpurun_out/lt.log; exit 1; }
tail -2 gpurun_out/lt.log
for cfg in ${CFGS:-1:0 2:0 3:0 1:2000 2:2000 3:2000}; do
k=${cfg%%:*}; sp=${cfg##*:}
KPSIM_POOL_SPIN_US=$sp KPSIM_LAUNCH_SUB=$k timeout -k 10 300 python bench.py --no-cpu-baseline --no-consolidation --no-topology --no-reserved --steps 20 --warmup 3 > gpurun_out/bl.json 2> gpurun_out/bl.err || { tail -5 gpurun_out/bl.err; exit 1; }
python3 -c "
import json; l=json.load(open('gpurun_out/bl.json'))['launch']; print('sub $k spin $sp', 'kernel %.3f busy %.3f call %.3f' % (l['kernel_ms'], l['device_busy_ms'], l['call_ms']), {k: round(v, 3) for k, v in l['call_phases_ms'].items()})"
done
