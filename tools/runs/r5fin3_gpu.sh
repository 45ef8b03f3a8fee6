#!/bin/bash
# round 5 final tree: the scale tests and the side-stream test after the side-stream change
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest -x -v --timeout 100 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "side_stream or native_fork" -p no:cacheprovider > gpurun_out/r5fin3_side.log 2>&1; rc=$?; echo "side rc $rc"; grep -E "FAILED|passed|failed" gpurun_out/r5fin3_side.log | tail -3; [ $rc -eq 0 ] || exit $rc
TAG=r5fin3 bash tools/runs/r5f2_gpu.sh
