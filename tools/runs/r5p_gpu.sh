#!/bin/bash
# round 5: the q log's drift at C3 for 32 / 64 / 128 epoch-chunks (ratings per item per chunk
# 6.7 / 3.4 / 1.7) beside the atomic schedule: does a per-item-per-chunk density rule hold?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/probes/qlog_chunks_exact_speed.py gpurun_out/r5p_probe.jsonl --no-u1 --chunks 24,32,64,128 > gpurun_out/r5p_probe.log 2>&1; rc=$?
echo "probe rc $rc"; cat gpurun_out/r5p_probe.jsonl; exit $rc
