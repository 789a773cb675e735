set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --spp 256 --steps 2 --warmup 1 --no-cpu-baseline --no-isolated > gpurun_out/bench_$tag.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['ms_extend_per_step'], d['ms_shade_per_step'], d['ms_finish_per_step'])"; }
run l1 RTAMD_LANES=1
run l2 RTAMD_LANES=2
run l3 RTAMD_LANES=3
run l4 RTAMD_LANES=4
run l2_d256 RTAMD_LANES=2 RTAMD_TAIL_DIV=256
run l3_d256 RTAMD_LANES=3 RTAMD_TAIL_DIV=256
run l2_32M RTAMD_LANES=2 RTAMD_MAX_PATHS=33554432
run l4_32M RTAMD_LANES=4 RTAMD_MAX_PATHS=33554432
