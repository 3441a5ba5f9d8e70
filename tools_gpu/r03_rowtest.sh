set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "row_items or chunked" 2>&1 | grep -E "PASS|FAIL|Error|assert|passed|failed" | tail -12
