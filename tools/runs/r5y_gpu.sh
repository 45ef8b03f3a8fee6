#!/bin/bash
# round 5: one long user chain alone (200k ratings over a 1M-item table): ns per rating of the
# SVD++ q-log kernel and helper-wave launch, and of the SVD checkpoint kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/probes/svdpp_long_chain.py gpurun_out/r5y_chain.jsonl > gpurun_out/r5y_chain.log 2>&1; rc=$?
echo "probe rc $rc"; cat gpurun_out/r5y_chain.jsonl; tail -3 gpurun_out/r5y_chain.log; exit $rc
