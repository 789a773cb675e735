#!/bin/bash
# A/B of the fused curve extend (RTAMD_CURVE_FUSE=1: every depth >= 1 in one launch) against one launch per
# depth (=0), C5 at SPP samples, variants interleaved ROUNDS times, extra bench args after them:
#   tools/ab_curve_fuse.sh TAG SPP ROUNDS [args]
set -o pipefail
TAG=${1:-abfuse}; SPP=${2:-8}; ROUNDS=${3:-2}
shift 3
O=gpurun_out/$TAG
mkdir -p $O
B="bench.py --scene curves --spp $SPP --steps 1 --warmup 1 --no-cpu-baseline --no-isolated $*"
for r in $(seq 1 $ROUNDS); do
  for F in 0 1; do
    RTAMD_CURVE_FUSE=$F timeout -k 10 600 python3 -u $B > $O/f${F}_r$r.log 2>&1 || { tail -5 $O/f${F}_r$r.log; exit 1; }
    echo "round $r fuse $F $(grep '^{' $O/f${F}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("ms_extend_per_step"))')"
  done
done
