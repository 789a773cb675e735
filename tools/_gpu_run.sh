set -o pipefail
O=gpurun_out/ab10
mkdir -p $O
python -c "import torch, numpy" || exit 1
B="timeout -k 10 100 python bench.py --no-cpu-baseline --no-isolated --spp 256 --steps 4"
run() { tag=$1; shift; env "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }; python -c "import json; d=json.loads([l for l in open('$O/$tag.log').read().splitlines() if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'], d['ms_finish_per_step'])"; }
run lds $B
run hbm RTAMD_FINISH_TREE_HBM=1 $B
run lds_b $B
run hbm_b RTAMD_FINISH_TREE_HBM=1 $B
run lds_l1 RTAMD_LANES=1 $B
run hbm_l1 RTAMD_LANES=1 RTAMD_FINISH_TREE_HBM=1 $B
