#!/bin/bash
# A/B of the lambertian shade's occupancy on C2 (256 spp, two lanes): base, leaf records from L2 instead of
# LDS (RTAMD_SHADE_LL=0), and a build capped at 4 waves per SIMD (rtamd/librtamd_w4.so, -DRT_SHADE_WAVES=4).
set -o pipefail
TAG=${1:-abshade}; ROUNDS=${2:-2}
O=gpurun_out/$TAG
mkdir -p $O
B="bench.py --spp 256 --steps 3 --warmup 1 --no-cpu-baseline --no-isolated"
cp scheme-raytrace_amd/rtamd/librtamd.so $O/base.so
one() { tag=$1; shift; env "$@" timeout -k 10 300 python3 -u $B > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
        echo "$tag $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
for r in $(seq 1 $ROUNDS); do
  cp $O/base.so scheme-raytrace_amd/rtamd/librtamd.so
  one base_r$r X=1
  one noll_r$r RTAMD_SHADE_LL=0
  cp scheme-raytrace_amd/rtamd/librtamd_w4.so scheme-raytrace_amd/rtamd/librtamd.so
  one w4_r$r X=1
  one w4noll_r$r RTAMD_SHADE_LL=0
done
cp $O/base.so scheme-raytrace_amd/rtamd/librtamd.so
rm -f $O/base.so
