#!/bin/bash
# round 5: the q log (fused fold, nt log stores) at scale -- the C5-shard 20-epoch RMSE test, then
# the full C5 on one GPU with its RMSE leg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -v -s --timeout 650 --timeout-method thread -m gpu tests/test_gpu_scale.py -k "qlog_e20" -p no:cacheprovider > gpurun_out/r5j_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r5j_pytest.log | tail -6
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 800 python3 -u bench.py --shape c5 --qlog --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 2 --warmup 1 --detail gpurun_out/r5j_c5full_qlog_detail.json > gpurun_out/r5j_c5full_qlog.json 2> gpurun_out/r5j_c5full_qlog.log; rc=$?
tail -3 gpurun_out/r5j_c5full_qlog.log; head -c 1500 gpurun_out/r5j_c5full_qlog.json; echo; exit $rc
