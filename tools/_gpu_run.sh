set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --spp 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$tag.log').read().strip().splitlines()[-1]); r=d['roofline_isolated']; print('$tag', d['value'], d['ms_per_step'], d['ms_extend_per_step'], d['ms_shade_per_step'], d['ms_finish_per_step'], r and r['frac'])"; }
run base_l1 RTAMD_LANES=1
run sw4_l1 RTAMD_LANES=1 RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_sw4.so
run sw5_l1 RTAMD_LANES=1 RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_sw5.so
