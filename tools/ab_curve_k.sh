#!/bin/bash
# A/B of the split curve extend's list capacity (RTAMD_CURVE_K) against the one-kernel curve extend, C5 at
# a few spp (one frame per variant), with the split's diagnostics (RTAMD_CURVE_DEBUG) on the first one.
#   usage: tools/ab_curve_k.sh TAG SPP "K1 K2 ..."
set -o pipefail
TAG=${1:-abk}; SPP=${2:-8}; KS=${3:-"8 16 32 64"}
O=gpurun_out/$TAG
mkdir -p $O
B="bench.py --scene curves --spp $SPP --steps 1 --warmup 1 --no-cpu-baseline --no-isolated"
RTAMD_CURVE_SPLIT=0 timeout -k 10 300 python3 -u $B > $O/old.log 2>&1 || exit 1
echo "old $(grep '^{' $O/old.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_extend_per_step"])')"
for K in $KS; do
  RTAMD_CURVE_SPLIT=1 RTAMD_CURVE_K=$K timeout -k 10 300 python3 -u $B > $O/k$K.log 2>&1 || exit 1
  RTAMD_CURVE_SPLIT=1 RTAMD_CURVE_K=$K RTAMD_CURVE_DEBUG=1 timeout -k 10 300 python3 -u $B --steps 1 --warmup 0 > $O/k${K}_dbg.log 2>&1 || exit 1
  echo "K=$K $(grep '^{' $O/k$K.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_extend_per_step"])') $(grep 'listed' $O/k${K}_dbg.log | head -3 | tr '\n' ' ')"
done
