#!/bin/bash
# round 5: the q log as the one-rank default where a chunk holds <= 10 ratings per item
# (auto_qlog) -- the C5 scale tests that name their schedule, then the full C5 on its default
# schedule (now the q log, fold indices ahead) with its RMSE leg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5q
timeout -k 10 1000 python -u -m pytest -v -s --timeout 900 --timeout-method thread -m gpu tests/test_gpu_scale.py -k "c5_shard or miniature or two_ranks_within" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "PASSED|FAILED|passed|failed|c5_u60000 E=20" gpurun_out/${tag}_pytest.log | tail -12
case $rc in 124|137|134|139) exit $rc;; esac
[ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python3 -u bench.py --shape c5 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 2 --warmup 1 --detail gpurun_out/${tag}_c5full_detail.json > gpurun_out/${tag}_c5full.json 2> gpurun_out/${tag}_c5full.log; rc=$?
tail -2 gpurun_out/${tag}_c5full.log; head -c 700 gpurun_out/${tag}_c5full.json; echo; exit $rc
