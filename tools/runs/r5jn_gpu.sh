#!/bin/bash
# round 5: the headline step's join variants (tools/probes/headline_join.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/probes/headline_join.py gpurun_out/r5jn_join.jsonl > gpurun_out/r5jn.log 2>&1; rc=$?
echo "rc $rc"; cat gpurun_out/r5jn_join.jsonl; tail -3 gpurun_out/r5jn.log; exit $rc
