#!/bin/bash
# Round-5 PMC profile sets for every benchmark scene (tools/profile_round.sh per scene), so each bench line
# carries traffic / valu / valu_issue from profiles/pmc/<scene>_{extend,shade}.json (kernel-hash stamped).
#   usage: tools/profile_scenes.sh TAG [SCENES]   (SCENES: a subset of "c2 c5 c3 c4 c4m", default all)
set -o pipefail
TAG=${1:-r05}
ONLY=${2:-"c2 c5 c3 c4 c4m"}
run() { name=$1; shift; case " $ONLY " in *" $name "*) ;; *) return 0;; esac; timeout -k 10 900 bash tools/profile_round.sh ${TAG}_$name "$@" > gpurun_out/prof_${TAG}_$name.log 2>&1 || { echo "profile $name failed"; tail -5 gpurun_out/prof_${TAG}_$name.log; exit 1; }; echo "profile $name ok"; }
mkdir -p gpurun_out
run c2
# C5 profiles the per-depth curve kernel the 256-spp configuration runs (a 4-spp frame would take the fused
# curve extend: depth-1 launches of <= 16M rays)
export RTAMD_CURVE_FUSE=0
run c5 --scene curves --spp 4
unset RTAMD_CURVE_FUSE
run c3 --scene cover_marble --spp 256
run c4 --scene cornell --nx 1024 --ny 1024 --spp 256
run c4m --scene cornell_mixture --nx 1024 --ny 1024 --spp 256
ls profiles/pmc/
