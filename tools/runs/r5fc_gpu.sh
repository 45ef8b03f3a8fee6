#!/bin/bash
# round 5 final tree: the C5 shard and the full C5 (10M x 1M x 990M, SVD++ K=128 fp32) on their
# default schedule (the q log, the shared-step chain), the full C5 with its E=20 RMSE leg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5fc
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; print('$1', 'value', r['value'], 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'rmse', (r.get('rmse') or {}).get('gpu'))"; }
timeout -k 10 300 python3 -u bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1 --detail gpurun_out/${tag}_c5q_d.json > gpurun_out/${tag}_c5q.json 2> gpurun_out/${tag}_c5q.log; rc=$?; show ${tag}_c5q; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 850 python3 -u bench.py --shape c5 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 2 --warmup 1 --detail gpurun_out/${tag}_c5full_d.json > gpurun_out/${tag}_c5full.json 2> gpurun_out/${tag}_c5full.log; rc=$?; show ${tag}_c5full; exit $rc
