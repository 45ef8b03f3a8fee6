#!/bin/bash
# round 5: what stretches C3's chains under full load (tools/probes/svdpp_c3_load.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/probes/svdpp_c3_load.py gpurun_out/r5ld_c3_load.jsonl > gpurun_out/r5ld.log 2>&1; rc=$?
echo "rc $rc"; cat gpurun_out/r5ld_c3_load.jsonl; tail -3 gpurun_out/r5ld.log; exit $rc
