set -o pipefail
O=gpurun_out/ab20
mkdir -p $O
python -c "import torch, numpy" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-isolated --steps 2"
run() { tag=$1; shift; env "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }; python -c "import json; d=json.loads([l for l in open('$O/$tag.log').read().splitlines() if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"; }
run d128 $B
run d256 RTAMD_TAIL_DIV=256 $B
run d128b $B
timeout -k 10 400 python bench.py > $O/bench_c2.log 2>&1 || exit 1
grep "^{" $O/bench_c2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['roofline_isolated']['frac'], d['roofline_shade_isolated']['frac'], d['cpu_baseline']['value'])"
