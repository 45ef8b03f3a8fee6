#!/bin/bash
# round 5: the driver's own GPU-test command on the final tree, in one process
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests/ -x -q -m gpu --timeout 1000 --timeout-method thread -p no:cacheprovider > gpurun_out/r5drv_pytest.log 2>&1; rc=$?
echo "rc $rc"; tail -4 gpurun_out/r5drv_pytest.log; exit $rc
