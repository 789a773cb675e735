set -o pipefail
O=gpurun_out/ab18
mkdir -p $O
python -c "import torch, numpy" || exit 1
B="timeout -k 10 100 python bench.py --no-cpu-baseline --no-isolated --spp 256 --steps 4"
run() { tag=$1; shift; env "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }; python -c "import json; d=json.loads([l for l in open('$O/$tag.log').read().splitlines() if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"; }
run base $B
run b1024 RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_b1024.so $B
run base2 $B
run b1024b RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_b1024.so $B
