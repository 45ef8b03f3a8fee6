#!/bin/bash
# round 5: C3 hot-row replica sweep (tools/probes/svdpp_c3_hot.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u tools/probes/svdpp_c3_hot.py gpurun_out/r5ht_c3_hot.jsonl > gpurun_out/r5ht.log 2>&1; rc=$?
echo "rc $rc"; cat gpurun_out/r5ht_c3_hot.jsonl; tail -3 gpurun_out/r5ht.log; exit $rc
