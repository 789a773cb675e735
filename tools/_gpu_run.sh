set -o pipefail
O=gpurun_out/ab4
mkdir -p $O
python -c "import torch, numpy" || exit 1
B="timeout -k 10 150 python bench.py --no-cpu-baseline --no-isolated --scene curves --spp 4 --steps 1 --warmup 1"
run() { tag=$1; shift; env "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }; python -c "import json; d=json.loads([l for l in open('$O/$tag.log').read().splitlines() if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'], d['segments_per_path'])"; }
run base RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_base.so $B
run half $B
run w3 RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_w3.so $B
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "curve or bezier" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
