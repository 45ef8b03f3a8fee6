#!/bin/bash
# round 5: SVD's exact-order default for small fits (deterministic=None) -- the u1 / configs[0]
# parity tests that name the schedule, smoke(), and the C5-shard q-log fold kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5l
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "configs0 or unbiased or log_mode or parallel_rmse or headline_configuration or batched_test or pickle or zero_epochs or test_metrics" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/${tag}_pytest.log | tail -40; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/${tag}_smoke.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${tag}_c5q -o run -- python3 $GRAFT_REPO_ROOT/bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1 --qlog > $GRAFT_REPO_ROOT/gpurun_out/${tag}_c5q.json 2> $GRAFT_REPO_ROOT/gpurun_out/${tag}_c5q.log; rc=$?
cd $GRAFT_REPO_ROOT; head -c 400 gpurun_out/${tag}_c5q.json; echo; f=$(ls gpurun_out/prof_${tag}_c5q/*/run_kernel_stats.csv gpurun_out/prof_${tag}_c5q/run_kernel_stats.csv 2>/dev/null | head -1); head -8 "$f"; exit $rc
