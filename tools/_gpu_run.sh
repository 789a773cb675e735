set -o pipefail
O=gpurun_out/ab17
mkdir -p $O
python -c "import torch, numpy" || exit 1
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-isolated --steps 2"
run() { tag=$1; shift; env "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }; python -c "import json; d=json.loads([l for l in open('$O/$tag.log').read().splitlines() if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"; }
run l2 $B
run l3 RTAMD_LANES=3 $B
run l4 RTAMD_LANES=4 $B
run l2b $B
