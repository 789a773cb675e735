#!/bin/bash
# A/B of two builds of librtamd (rtamd/librtamd.so = new, rtamd/librtamd_base.so = base), variants
# interleaved: tools/ab_so.sh TAG ROUNDS "bench args"
set -o pipefail
TAG=${1:-abso}; ROUNDS=${2:-2}; ARGS=${3:-"--scene curves --spp 8"}
O=gpurun_out/$TAG
mkdir -p $O
R=scheme-raytrace_amd/rtamd
cp $R/librtamd.so $O/new.so
B="bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline --no-isolated"
one() { tag=$1; timeout -k 10 600 python3 -u $B > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; cp $O/new.so $R/librtamd.so; exit 1; }
        echo "$tag $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
for r in $(seq 1 $ROUNDS); do
  cp $R/librtamd_base.so $R/librtamd.so; one base_r$r
  cp $O/new.so $R/librtamd.so; one new_r$r
done
cp $O/new.so $R/librtamd.so
rm -f $O/new.so
