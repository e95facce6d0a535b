set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-launch --no-topology --no-reserved --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bcq.json 2> gpurun_out/bcq.err || { tail -5 gpurun_out/bcq.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bcq.json'))
for l in ('consolidation','consolidation_replace'): c=d[l]; print(l, c['candidates_per_s'], c['value'], c['kernel_ms_rank0'])"
