#!/bin/bash
# round 5: the next chunk's <p^2> summed in fixed-range parts from 64k users (ABI 933) and the
# replay's non-temporal row gathers -- the whole parity file, then the C5 shard and the full C5 on
# their default schedule (the q log) with the new sum
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5t
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; ph=rl.get('phases_gpu_ms',{}); print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'epoch', ph.get('epoch_kernel_ms'), 'replay', ph.get('replay_ms'), 'fold', ph.get('fold_sync_ms'), 'rmse', (r.get('rmse') or {}).get('gpu'))"; }
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_abi.py -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed|past_64k|fixed_parts" gpurun_out/${tag}_pytest.log | tail -12; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1 --detail gpurun_out/${tag}_c5q_d.json > gpurun_out/${tag}_c5q.json 2> gpurun_out/${tag}_c5q.log; rc=$?; show ${tag}_c5q; fatal $rc
timeout -k 10 300 python3 -u bench.py --shape c4 --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 5 --warmup 2 --detail gpurun_out/${tag}_c4_d.json > gpurun_out/${tag}_c4.json 2> gpurun_out/${tag}_c4.log; rc=$?; show ${tag}_c4; fatal $rc
timeout -k 10 800 python3 -u bench.py --shape c5 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 2 --warmup 1 --detail gpurun_out/${tag}_c5full_d.json > gpurun_out/${tag}_c5full.json 2> gpurun_out/${tag}_c5full.log; rc=$?; show ${tag}_c5full; exit $rc
