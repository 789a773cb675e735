set -o pipefail
O=gpurun_out/r01j
mkdir -p $O
python -c "import torch, numpy" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile_round.sh r01j || exit 1
RTAMD_LANES=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r01j/kt_l1 -o kt -- python3 bench.py --spp 256 --steps 1 --warmup 0 --no-cpu-baseline --no-isolated > gpurun_out/prof_r01j/kt_l1.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 1; }
timeout -k 10 300 python bench.py --scene cover_marble --spp 256 --no-cpu-baseline > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --scene cornell --nx 1024 --ny 1024 --spp 512 > $O/bench_c4.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --scene cornell_mixture --nx 1024 --ny 1024 --spp 512 --no-cpu-baseline > $O/bench_c4m.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --scene curves --spp 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit 1
for f in $O/bench_*.log; do python -c "import json,sys; d=json.loads([l for l in open('$f').read().splitlines() if l.startswith('{')][-1]); c=d.get('cpu_baseline') or {}; r=d.get('roofline_isolated') or {}; sh=d.get('roofline_shade_isolated') or {}; print('$f', d['value'], d['ms_per_step'], d['segments_per_path'], c.get('value'), r.get('frac'), (d.get('roofline') or {}).get('frac'), sh.get('frac'), d['samples_per_s'])"; done
