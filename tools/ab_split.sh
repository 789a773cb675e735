#!/bin/bash
# Round-5 A/B of the split curve extend's knobs (C5 at a few spp), then its kernel profile.
#   usage: tools/ab_split.sh TAG SPP
set -o pipefail
TAG=${1:-abs}; SPP=${2:-8}
O=gpurun_out/$TAG
mkdir -p $O
L=scheme-raytrace_amd/rtamd
timeout -k 10 600 python3 tools/ab_lib.py --scene curves --spp $SPP --rounds 2 \
  old:$L/librtamd.so:RTAMD_CURVE_SPLIT=0 \
  k32:$L/librtamd.so:RTAMD_CURVE_SPLIT=1 \
  k16:$L/librtamd.so:RTAMD_CURVE_SPLIT=1,RTAMD_CURVE_K=16 \
  k8:$L/librtamd.so:RTAMD_CURVE_SPLIT=1,RTAMD_CURVE_K=8 \
  p32:$L/librtamd.so:RTAMD_CURVE_SPLIT=1,RTAMD_TRAV_PERSIST=1 \
  p16:$L/librtamd.so:RTAMD_CURVE_SPLIT=1,RTAMD_TRAV_PERSIST=1,RTAMD_CURVE_K=16 \
  if2p16:$L/librtamd_if2.so:RTAMD_CURVE_SPLIT=1,RTAMD_TRAV_PERSIST=1,RTAMD_CURVE_K=16 \
  if4p32:$L/librtamd_if4.so:RTAMD_CURVE_SPLIT=1,RTAMD_TRAV_PERSIST=1 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep "round 1" $O/ab.log; tail -1 $O/ab.log
for v in "RTAMD_CURVE_K=32" "RTAMD_CURVE_K=16" "RTAMD_CURVE_K=16 RTAMD_TRAV_PERSIST=1"; do
  env RTAMD_CURVE_SPLIT=1 RTAMD_CURVE_DEBUG=1 $v timeout -k 10 300 python3 -u bench.py --scene curves --spp $SPP --steps 1 --warmup 0 --no-cpu-baseline --no-isolated > "$O/dbg_${v// /_}.log" 2>&1 || exit 1
  echo "$v: $(grep 'listed' "$O/dbg_${v// /_}.log" | head -2 | tr '\n' ' ')"
done
export TMPDIR=/tmp
RTAMD_CURVE_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_split -o kt -- python3 bench.py --scene curves --spp $SPP --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events > $O/prof_split.log 2>&1 || exit 1
RTAMD_CURVE_SPLIT=1 RTAMD_TRAV_PERSIST=1 RTAMD_CURVE_K=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_split_p16 -o kt -- python3 bench.py --scene curves --spp $SPP --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events > $O/prof_split_p16.log 2>&1 || exit 1
echo done
