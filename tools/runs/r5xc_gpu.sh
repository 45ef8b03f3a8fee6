#!/bin/bash
# round 5: C3 heavy chains on one XCD (tools/probes/svdpp_c3_xcd.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/probes/svdpp_c3_xcd.py gpurun_out/r5xc_c3_xcd.jsonl > gpurun_out/r5xc.log 2>&1; rc=$?
echo "rc $rc"; cat gpurun_out/r5xc_c3_xcd.jsonl; tail -3 gpurun_out/r5xc.log; exit $rc
