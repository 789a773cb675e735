#!/bin/bash
# bench.py's C2 line with and without the per-launch HIP events in the timed frames, interleaved
set -o pipefail
TAG=${1:-abpe}; ROUNDS=${2:-3}
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for v in ev noev; do
    X=""; [ $v = noev ] && X="--no-profile-events"
    timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-isolated $X > $O/${v}_r$r.log 2>&1 || { tail -5 $O/${v}_r$r.log; exit 1; }
    echo "round $r $v $(grep '^{' $O/${v}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
