#!/bin/bash
# A/B of the exact-libm cost on C2 (RT_OPT_EXACT_LIBM auto vs exact) for library builds given as name:path.
#   usage: tools/ab_libm.sh TAG SPP name:lib ...
set -o pipefail
TAG=${1:-abl}; SPP=${2:-256}; shift 2
O=gpurun_out/$TAG
mkdir -p $O
for round in 0 1; do
  for v in "$@"; do
    name=${v%%:*}; lib=${v#*:}
    for mode in auto exact; do
      RTAMD_LIB=$PWD/$lib timeout -k 10 300 python3 -u bench.py --spp $SPP --steps 2 --warmup 1 --no-cpu-baseline --no-isolated --exact-libm $mode > $O/${name}_${mode}_$round.log 2>&1 || exit 1
      echo "round $round $name $mode $(grep '^{' $O/${name}_${mode}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_shade_per_step"])')"
    done
  done
done
