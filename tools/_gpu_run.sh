set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --spp 256 --steps 2 --warmup 1 --no-cpu-baseline --no-isolated > gpurun_out/bench_$tag.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['ms_extend_per_step'], d['ms_shade_per_step'], d['ms_finish_per_step'])"; }
L=scheme-raytrace_amd/rtamd
run rf16 RTAMD_LANES=1
run rf32 RTAMD_LANES=1 RTAMD_LIB=$L/librtamd_rf32.so
run rf48 RTAMD_LANES=1 RTAMD_LIB=$L/librtamd_rf48.so
run rf64 RTAMD_LANES=1 RTAMD_LIB=$L/librtamd_rf64.so
