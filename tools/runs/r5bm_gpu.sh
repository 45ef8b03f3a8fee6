#!/bin/bash
# round 5: fp32 headline engine instances (tools/probes/headline_bimodal.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/probes/headline_bimodal.py gpurun_out/r5bm_join.jsonl > gpurun_out/r5bm.log 2>&1; rc=$?
echo "rc $rc"; cat gpurun_out/r5bm_join.jsonl; tail -3 gpurun_out/r5bm.log; exit $rc
