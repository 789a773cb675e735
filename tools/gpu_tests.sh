#!/bin/bash
# pytest -m gpu on the GPU box (from the repo root), log under gpurun_out/TAG.
#   usage: tools/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-tests}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|rms=|pooled|passed|failed" $O/pytest_gpu.log | tail -40
exit $rc
