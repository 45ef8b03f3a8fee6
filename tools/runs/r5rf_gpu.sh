#!/bin/bash
# round 5: the fold inside the replays (engine option replay_fold, mf_launch_fold) -- its parity
# test and the other split-chunk tests, then the headline step with and without it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "replay_fold or native_fork or headline_configuration or checkpoint_rows or narrow" -p no:cacheprovider > gpurun_out/r5rf_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/r5rf_pytest.log | tail -8; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probes/headline_join.py gpurun_out/r5rf_join.jsonl > gpurun_out/r5rf_probe.log 2>&1; rc=$?; echo "probe rc $rc"; cat gpurun_out/r5rf_join.jsonl; exit $rc
