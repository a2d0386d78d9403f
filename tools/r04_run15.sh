#!/bin/bash
# r04: Bloom filters past the Redis offset limit (|size| > 2^32) + the Bloom / lifecycle / node suites
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_lifecycle_gpu.py tests/test_bloom_gpu.py tests/test_node_gpu.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests15.log" 2>&1
rc=$?
echo "tests rc=$rc"
grep -E "passed|failed|Error|error" "$O/gpu_tests15.log" | tail -15
exit $rc
