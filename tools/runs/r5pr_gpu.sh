#!/bin/bash
# round 5: join variants and replay piece length (tools/probes/headline_join.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/probes/headline_join.py gpurun_out/r5pr_join.jsonl > gpurun_out/r5pr.log 2>&1; rc=$?
echo "rc $rc"; cat gpurun_out/r5pr_join.jsonl; tail -3 gpurun_out/r5pr.log; exit $rc
