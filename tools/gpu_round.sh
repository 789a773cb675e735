#!/bin/bash
# One GPU pass of the tree (run on the GPU box from the repo root), logs under gpurun_out/TAG:
#   pytest -m gpu, smoke(), bench C2 (default line), bench C5 (256 spp), rocprof + PMC profile sets of both.
#   usage: tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_c2.log 2>&1 || { echo "bench C2 failed"; tail -20 $O/bench_c2.log; exit 1; }
timeout -k 10 500 python -u bench.py --scene curves --spp 256 --steps 1 --warmup 1 > $O/bench_c5.log 2>&1 || { echo "bench C5 failed"; tail -20 $O/bench_c5.log; exit 1; }
for s in c2 c5; do
  grep '^{' $O/bench_$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; f=d.get('roofline_frame') or {}; p=d.get('parity') or {}; q=d.get('parity_frame') or {}; print('$s', d['value'], d['ms_per_step'], 'roof', r.get('frac'), 'frame', f.get('frac'), 'parity', p.get('rms_vs_oracle'), p.get('pixels_gt_1e-9'), 'frame_rows', q.get('rms_vs_oracle'), q.get('pixels_gt_1e-9'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
timeout -k 10 600 bash tools/profile_round.sh ${TAG}_c2 > $O/prof_c2.log 2>&1 || { echo "profile C2 failed"; tail -5 $O/prof_c2.log; exit 1; }
mkdir -p $O/pmc_c2 && cp profiles/pmc/*.json $O/pmc_c2/
timeout -k 10 600 bash tools/profile_round.sh ${TAG}_c5 --scene curves --spp 4 > $O/prof_c5.log 2>&1 || { echo "profile C5 failed"; tail -5 $O/prof_c5.log; exit 1; }
echo done
