set -o pipefail
mkdir -p gpurun_out/r01f
O=gpurun_out/r01f
timeout -k 10 400 python bench.py > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 1; }
timeout -k 10 300 python bench.py --scene cover_marble --spp 256 --no-cpu-baseline > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --scene cornell --nx 1024 --ny 1024 --spp 512 > $O/bench_c4.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --scene cornell_mixture --nx 1024 --ny 1024 --spp 512 --no-cpu-baseline > $O/bench_c4m.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --scene curves --spp 16 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit 1
for f in $O/bench_*.log; do python -c "import json,sys; d=json.loads([l for l in open('$f').read().splitlines() if l.startswith('{')][-1]); c=d.get('cpu_baseline') or {}; r=d.get('roofline_isolated') or {}; print('$f', d['value'], d['ms_per_step'], d['segments_per_path'], c.get('value'), r.get('frac'))"; done
