#!/bin/bash
# A/B of the render lanes for the curve scene (C5), variants interleaved: tools/ab_lanes_c5.sh TAG SPP ROUNDS
set -o pipefail
TAG=${1:-ablanes}; SPP=${2:-32}; ROUNDS=${3:-2}
O=gpurun_out/$TAG
mkdir -p $O
B="bench.py --scene curves --spp $SPP --steps 2 --warmup 1 --no-cpu-baseline --no-isolated"
for r in $(seq 1 $ROUNDS); do
  for N in 1 2; do
    timeout -k 10 300 python3 -u $B --lanes $N > $O/l${N}_r$r.log 2>&1 || { tail -5 $O/l${N}_r$r.log; exit 1; }
    echo "round $r lanes $N $(grep '^{' $O/l${N}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
