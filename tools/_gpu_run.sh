set -o pipefail
O=gpurun_out/prof_final
mkdir -p $O
python -c "import torch, numpy" || exit 1
RTAMD_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_l1_full -o kt -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-isolated > $O/kt_l1_full.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_full -o kt -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-isolated > $O/kt_full.log 2>&1 || exit 1
grep "^{" $O/kt_l1_full.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_ms'])"
