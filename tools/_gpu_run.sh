set -o pipefail
O=gpurun_out/shade
mkdir -p $O
python -c "import torch, numpy" || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --spp 256 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/b.log').read().splitlines() if l.startswith('{')][-1]); print(d['value'], json.dumps(d['roofline_shade_isolated']), json.dumps(d['roofline_isolated']))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
