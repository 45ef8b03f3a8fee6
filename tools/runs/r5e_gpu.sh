#!/bin/bash
# round 5: the fused q-log fold with hot-item pieces -- parity, then the C5 shard timing with a
# kernel trace; the XCD dispatch-check test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r5e}
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ext.py -k "qlog or dispatch or helper_ring" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/${tag}_pytest.log | tail -20; fatal $rc
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline'].get('phases_gpu_ms',{}); print('$1', r['config']['workload'][-50:], 'ms/step', round(r['ms_per_step'],3), ph)"; }
B5="python3 -u bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${tag}_c5q -o run -- $B5 --qlog --detail gpurun_out/${tag}_c5q_detail.json > gpurun_out/${tag}_c5q.json 2> gpurun_out/${tag}_c5q.log; rc=$?; show ${tag}_c5q; fatal $rc
head -14 gpurun_out/prof_${tag}_c5q/run_kernel_stats.csv | cut -c1-150
