#!/bin/bash
# A/B of render-lane stream priorities (RTAMD_LANE_PRIO 0 / 1 / 2) on C2, variants interleaved
set -o pipefail
TAG=${1:-abprio}; ROUNDS=${2:-2}; ARGS=${3:-""}
O=gpurun_out/$TAG
mkdir -p $O
B="bench.py $ARGS --steps 3 --warmup 1 --no-cpu-baseline --no-isolated"
for r in $(seq 1 $ROUNDS); do
  for P in 0 1 2; do
    RTAMD_LANE_PRIO=$P timeout -k 10 300 python3 -u $B > $O/p${P}_r$r.log 2>&1 || { tail -5 $O/p${P}_r$r.log; exit 1; }
    echo "round $r prio $P $(grep '^{' $O/p${P}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
