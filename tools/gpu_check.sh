#!/bin/bash
# One GPU check of the tree (run on the GPU box from the repo root):
#   pytest -m gpu, smoke(), and the default bench line.   usage: tools/gpu_check.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_c2.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_c2.log; exit 1; }
grep '^{' $O/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('rms_vs_oracle'), d.get('max_abs'), d.get('pixels_gt_1e-9'), d['roofline']['frac'], (d.get('roofline_frame') or {}).get('frac'), (d.get('parity_frame') or {}).get('rms_vs_oracle'), d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
