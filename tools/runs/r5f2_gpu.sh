#!/bin/bash
# round 5 final rehearsal, part 2: tests/test_gpu_scale.py (C4 / C5 shard / C5@8 schedule / C5
# miniature / big tables) on the final tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1150 python -u -m pytest -v -s --timeout 1000 --timeout-method thread -m gpu tests/test_gpu_scale.py -p no:cacheprovider > gpurun_out/${TAG:-r5f}_scale.log 2>&1; rc=$?; echo "scale rc $rc"; grep -E "PASSED|FAILED|passed|failed|E=20" gpurun_out/${TAG:-r5f}_scale.log | tail -20; exit $rc
