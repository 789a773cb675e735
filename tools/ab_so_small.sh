#!/bin/bash
# A/B of two builds (rtamd/librtamd.so = new, rtamd/librtamd_base.so = base) on small frames of C2's scene
# (tools/small_frames.py) and on bench.py lines: tools/ab_so_small.sh TAG "SPPS" "bench args"
set -o pipefail
TAG=${1:-absmall}; SPPS=${2:-"1 4"}; BARGS=${3:-""}
O=gpurun_out/$TAG
mkdir -p $O
R=scheme-raytrace_amd/rtamd
cp $R/librtamd.so $O/new.so
for v in base new base new; do
  if [ $v = base ]; then cp $R/librtamd_base.so $R/librtamd.so; else cp $O/new.so $R/librtamd.so; fi
  for s in $SPPS; do
    FRAMES=20 timeout -k 10 300 python -u tools/small_frames.py $s 0 > $O/${v}_spp$s.log 2>&1 || { tail -5 $O/${v}_spp$s.log; cp $O/new.so $R/librtamd.so; exit 1; }
    echo "$v spp $s: $(grep 'round 1' $O/${v}_spp$s.log)"
  done
  if [ -n "$BARGS" ]; then
    timeout -k 10 300 python3 -u bench.py $BARGS --no-cpu-baseline --no-isolated > $O/${v}_bench.log 2>&1 || { tail -5 $O/${v}_bench.log; cp $O/new.so $R/librtamd.so; exit 1; }
    echo "$v bench: $(grep '^{' $O/${v}_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  fi
done
cp $O/new.so $R/librtamd.so
rm -f $O/new.so
