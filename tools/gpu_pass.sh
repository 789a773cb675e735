#!/bin/bash
# One GPU pass (run on the GPU box from the repo root), logs under gpurun_out/TAG:
#   pytest -m gpu (all tests; a test failure does not stop the pass, a crash / time limit does),
#   smoke(), then each bench command given after the tag (quoted), e.g.
#   tools/gpu_pass.sh r05b "bench.py" "bench.py --scene curves --spp 256 --steps 1"
# Every GPU step has its own time limit; after an abort, a segfault or a limit nothing else runs.
set -o pipefail
TAG=${1:-pass}
shift || true
O=gpurun_out/$TAG
mkdir -p $O
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }      # 0 passed, 1 = some tests failed (not a crash)
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
  rc=$?
  grep -E "passed|failed" $O/pytest_gpu.log | tail -1
  grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20
  ok $rc || { echo "pytest rc=$rc: stopping"; tail -20 $O/pytest_gpu.log; exit $rc; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
i=0
for cmd in "$@"; do
  i=$((i + 1))
  timeout -k 10 900 python -u $cmd > $O/bench_$i.log 2>&1
  rc=$?
  echo "bench $i ($cmd): rc=$rc"
  grep '^{' $O/bench_$i.log | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    if d.get('mode') == 'shard_balance':
        print('balance', d['config'], d['frame_ms'], {k: (v['ms_max_over_mean'], v['predicted_efficiency']) for k, v in d['partitions'].items()})
        continue
    r = d.get('roofline') or {}; f = d.get('roofline_frame') or {}; p = d.get('parity') or {}; q = d.get('parity_frame') or {}
    print(d['value'], d['ms_per_step'], 'roof', r.get('frac'), 'traffic', r.get('traffic'), 'frame', f.get('frac'), 'parity', p.get('rms_vs_oracle'), p.get('pixels_gt_1e-9'), 'frame_rows', q.get('rms_vs_oracle'), q.get('pixels_gt_1e-9'), {k: (v.get('rms_vs_oracle'), v.get('pixels_gt_1e-9')) for k, v in d.items() if k.startswith('parity_frame_')}, 'commit', d.get('scene_commit'))
"
  [ $rc -eq 0 ] || { tail -20 $O/bench_$i.log; exit $rc; }
done
echo done
