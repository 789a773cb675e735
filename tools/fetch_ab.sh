#!/bin/bash
# FETCH_SIZE of the curve kernel, base vs new build (C5 at 4 spp, one launch per depth): tools/fetch_ab.sh TAG
set -o pipefail
TAG=${1:-fetchab}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
R=scheme-raytrace_amd/rtamd
cp $R/librtamd.so $O/new.so
export TMPDIR=/tmp RTAMD_CURVE_FUSE=0
for v in base new; do
  if [ $v = base ]; then cp $R/librtamd_base.so $R/librtamd.so; else cp $O/new.so $R/librtamd.so; fi
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/$v -o f -- python3 bench.py --scene curves --spp 4 --steps 1 --warmup 0 --no-cpu-baseline --no-isolated --no-profile-events > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; cp $O/new.so $R/librtamd.so; exit 1; }
  echo "$v ok"
done
cp $O/new.so $R/librtamd.so
rm -f $O/new.so
