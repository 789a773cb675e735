#!/bin/bash
# The fused curve extend's finish batch (RTAMD_FUSE_BATCH) against one launch per depth, C5 at SPP samples:
#   tools/ab_fuse_batch.sh TAG SPP "BATCHES" [args]
set -o pipefail
TAG=${1:-abfb}; SPP=${2:-32}; BS=${3:-"20 32 48"}
shift 3
O=gpurun_out/$TAG
mkdir -p $O
B="bench.py --scene curves --spp $SPP --steps 1 --warmup 1 --no-cpu-baseline --no-isolated $*"
one() { tag=$1; shift; env "$@" timeout -k 10 600 python3 -u $B > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
        echo "$tag $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
one unfused RTAMD_CURVE_FUSE=0
for b in $BS; do one fused_b$b RTAMD_CURVE_FUSE=1 RTAMD_FUSE_BATCH=$b; done
