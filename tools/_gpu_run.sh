set -o pipefail
O=gpurun_out/tests
mkdir -p $O
python -c "import torch, numpy" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -k "wavefront_matches_tail or curve_kernels_bitwise" > $O/pytest_wf.log 2>&1; echo rc=$?; grep -E "PASSED|FAILED|Error|assert" $O/pytest_wf.log | head -40; tail -3 $O/pytest_wf.log
