set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 90 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log | cut -c1-300; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --spp 256 --steps 2 --warmup 1 --no-cpu-baseline --no-isolated > gpurun_out/bench_$tag.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['ms_extend_per_step'], d['ms_shade_per_step'], d['ms_finish_per_step'])"; }
L=scheme-raytrace_amd/rtamd
run pf_l1 RTAMD_LANES=1
run cw5_l1 RTAMD_LANES=1 RTAMD_LIB=$L/librtamd_cw5.so
run pf X=1
