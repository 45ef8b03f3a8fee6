#!/bin/bash
# round 5: is C3 bound by its heaviest chains?  One epoch of the fold vs its 1 / 8 / 64 heaviest users alone
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/probes/svdpp_c3_chain.py gpurun_out/r5c3_chain.jsonl > gpurun_out/r5c3_chain.log 2>&1; rc=$?; cat gpurun_out/r5c3_chain.jsonl; tail -2 gpurun_out/r5c3_chain.log; exit $rc
