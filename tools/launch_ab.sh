#!/bin/bash
# GPU-box A/B of kp_launch_select's host/device pipeline: launch parity tests, then the launch leg of bench.py with
# 1..4 sub-batches (KPSIM_LAUNCH_SUB) — kernel time, call time and host phases per setting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_launch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lt.log 2>&1 || { tail -30 gpurun_out/lt.log; exit 1; }
tail -2 gpurun_out/lt.log
for k in ${SUBS:-1 2 3 4}; do
KPSIM_LAUNCH_SUB=$k timeout -k 10 300 python bench.py --no-cpu-baseline --no-consolidation --no-topology --no-reserved --steps 10 --warmup 3 > gpurun_out/bl$k.json 2> gpurun_out/bl$k.err || { tail -5 gpurun_out/bl$k.err; exit 1; }
python3 -c "
import json; l=json.load(open('gpurun_out/bl$k.json'))['launch']; print($k, l['sub_batches'], 'kernel %.3f call %.3f' % (l['kernel_ms'], l['call_ms']), l['call_phases_ms'])"
done
