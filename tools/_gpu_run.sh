set -o pipefail
O=gpurun_out/ab13
mkdir -p $O
python -c "import torch, numpy" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-isolated --steps 2"
run() { tag=$1; shift; env "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }; python -c "import json; d=json.loads([l for l in open('$O/$tag.log').read().splitlines() if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"; }
run base RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_base.so $B
run new $B
run base_b RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_base.so $B
run new_b $B
run c4_base RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_base.so $B --scene cornell --nx 1024 --ny 1024 --spp 512
run c4_new $B --scene cornell --nx 1024 --ny 1024 --spp 512
run s256_base RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_base.so $B --spp 256
run s256_new $B --spp 256
