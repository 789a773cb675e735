set -o pipefail
O=gpurun_out/ab8
mkdir -p $O
python -c "import torch, numpy" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
B="timeout -k 10 100 python bench.py --no-cpu-baseline --no-isolated --spp 256 --steps 4"
run() { tag=$1; shift; env "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }; python -c "import json; d=json.loads([l for l in open('$O/$tag.log').read().splitlines() if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"; }
run base RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_base.so $B
run regen $B
run base_b RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_base.so $B
run regen_b $B
run base_l1 RTAMD_LANES=1 RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_base.so $B
run regen_l1 RTAMD_LANES=1 $B
