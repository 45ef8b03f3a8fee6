#!/bin/bash
# round 5: the fused SVD++ q-log fold -- parity (qlog tests, fused and not), then the C5 shard
# (1.25M users, 123M ratings, SVD++ K=128 fp32, 16 chunks) with the q log (fused) vs the atomic
# schedule, a kernel trace of the fused run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r5c}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 240 --timeout-method thread -k "qlog" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" gpurun_out/${tag}_pytest.log | tail -3; [ $rc -eq 0 ] || { tail -30 gpurun_out/${tag}_pytest.log; exit $rc; }
B="python3 -u bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1"
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; print('$1', r['config']['workload'][-60:], round(r['ms_per_step'],2), ph)"; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${tag}_qlog -o run -- $B --qlog --detail gpurun_out/${tag}_qlog_detail.json > gpurun_out/${tag}_qlog.json 2> gpurun_out/${tag}_qlog.log || exit $?; show ${tag}_qlog
head -12 gpurun_out/prof_${tag}_qlog/run_kernel_stats.csv | cut -c1-120
timeout -k 10 300 $B --detail gpurun_out/${tag}_atomic_detail.json > gpurun_out/${tag}_atomic.json 2> gpurun_out/${tag}_atomic.log || exit $?; show ${tag}_atomic
