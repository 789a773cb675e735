#!/bin/bash
# Bench lines for the other BASELINE configurations (run on the GPU box from the repo root):
#   C3 cover_marble 1920x1080x1024, C4 cornell 1024x1024x4096 (+ the f2 mixture), C5 curves 1920x1080x256.
#   usage: tools/bench_scenes.sh TAG [scene ...]
set -o pipefail
TAG=${1:-scenes}
shift || true
O=gpurun_out/$TAG
mkdir -p $O
SC=${@:-cover_marble cornell cornell_mixture curves}
for s in $SC; do
  case $s in
    cornell|cornell_mixture) A="--nx 1024 --ny 1024 --spp 4096 --steps 1 --warmup 1" ;;
    curves) A="--spp 256 --steps 1 --warmup 1" ;;
    *) A="--steps 1 --warmup 1" ;;
  esac
  timeout -k 10 900 python -u bench.py --scene $s $A > $O/bench_$s.log 2>&1 || { echo "bench $s failed"; tail -20 $O/bench_$s.log; exit 1; }
  grep '^{' $O/bench_$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d.get('parity') or {}; print(d['config']['workload'], d['value'], d['ms_per_step'], p.get('rms_vs_oracle'), p.get('pixels_gt_1e-9'), (d.get('roofline') or {}).get('frac'), (d.get('roofline_frame') or {}).get('frac'), (d.get('parity_frame') or {}).get('rms_vs_oracle'), (d.get('parity_frame') or {}).get('pixels_gt_1e-9'))"
done
