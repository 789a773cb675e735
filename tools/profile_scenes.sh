#!/bin/bash
# PMC profile sets for every benchmark scene (tools/profile_round.sh per scene), so each bench line
# carries traffic / valu / valu_issue from profiles/pmc/<scene>_{extend,shade}.json (kernel-hash stamped).
#   usage: tools/profile_scenes.sh TAG [SCENES]   (SCENES: a subset of "c2 c5 c3 c4 c4m", default all)
set -o pipefail
TAG=${1:-r05}
ONLY=${2:-"c2 c5 c3 c4 c4m"}
run() { name=$1; shift; case " $ONLY " in *" $name "*) ;; *) return 0;; esac; timeout -k 10 900 bash tools/profile_round.sh ${TAG}_$name "$@" > gpurun_out/prof_${TAG}_$name.log 2>&1 || { echo "profile $name failed"; tail -5 gpurun_out/prof_${TAG}_$name.log; exit 1; }; echo "profile $name ok"; }
mkdir -p gpurun_out
run c2
# every scene at its bench configuration (round 6: bench.py's load_pmc requires the profiled frame to be
# the benchmarked one, so C5's counters come from its 256-spp schedule — per-depth launches, then fused)
run c5 --scene curves --spp 256
run c3 --scene cover_marble
run c4 --scene cornell --nx 1024 --ny 1024 --spp 4096
run c4m --scene cornell_mixture --nx 1024 --ny 1024 --spp 4096
ls profiles/pmc/
