set -o pipefail
O=gpurun_out/final2
mkdir -p $O
python -c "import torch, numpy" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 1; }
timeout -k 10 300 python bench.py --scene cover_marble --spp 256 --no-cpu-baseline > $O/bench_c3.log 2>&1 || exit 1
for f in $O/bench_*.log; do python -c "import json,sys; d=json.loads([l for l in open('$f').read().splitlines() if l.startswith('{')][-1]); c=d.get('cpu_baseline') or {}; r=d.get('roofline_isolated') or {}; sh=d.get('roofline_shade_isolated') or {}; print('$f', d['value'], d['ms_per_step'], c.get('value'), r.get('frac'), (d.get('roofline') or {}).get('frac'), sh.get('frac'), d['samples_per_s'])"; done
