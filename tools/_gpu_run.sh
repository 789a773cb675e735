set -o pipefail
O=gpurun_out/ab16
mkdir -p $O
python -c "import torch, numpy" || exit 1
B="timeout -k 10 100 python bench.py --no-cpu-baseline --no-isolated --spp 256 --steps 4"
run() { tag=$1; shift; env "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }; python -c "import json; d=json.loads([l for l in open('$O/$tag.log').read().splitlines() if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"; }
L=scheme-raytrace_amd/rtamd
run base $B
run s5 RTAMD_LIB=$L/librtamd_s5.so $B
run s6 RTAMD_LIB=$L/librtamd_s6.so $B
run base2 $B
