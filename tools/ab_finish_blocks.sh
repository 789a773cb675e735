#!/bin/bash
# The tail kernel's grid (RTAMD_FINISH_BLOCKS) on small frames of C2's scene (tools/small_frames.py):
#   tools/ab_finish_blocks.sh TAG SPP "GRIDS"
set -o pipefail
TAG=${1:-abfb}; SPP=${2:-1}; GS=${3:-"512 1024 2048"}
O=gpurun_out/$TAG
mkdir -p $O
for g in $GS; do
  RTAMD_FINISH_BLOCKS=$g FRAMES=${FRAMES:-20} timeout -k 10 300 python -u tools/small_frames.py $SPP 0 > $O/spp${SPP}_g$g.log 2>&1 || { tail -5 $O/spp${SPP}_g$g.log; exit 1; }
  echo "grid $g: $(grep 'round 1' $O/spp${SPP}_g$g.log)"
done
