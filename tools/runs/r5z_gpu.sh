#!/bin/bash
# round 5: the SVD++ body's item biases by one per-lane gather per bank (SB: fp32 K=128) -- the
# SVD++ parity tests, then the C5 shard on the q log (default) and the atomic schedule, and C3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5z
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; ph=rl.get('phases_gpu_ms',{}); print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'epoch', ph.get('epoch_kernel_ms'), 'fold', ph.get('fold_sync_ms'), 'svdpp_c3', (r.get('svdpp_c3') or {}).get('f32_ms'))"; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ext.py -k "svdpp" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed" gpurun_out/${tag}_pytest.log | tail -6; fatal $rc; [ $rc -eq 0 ] || exit $rc
for q in 1 0; do
  timeout -k 10 300 python3 -u bench.py --shape c5 --users 1250000 --qlog $q --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1 --detail gpurun_out/${tag}_c5q${q}_d.json > gpurun_out/${tag}_c5q${q}.json 2> gpurun_out/${tag}_c5q${q}.log; rc=$?; show ${tag}_c5q${q}; fatal $rc
done
timeout -k 10 300 python3 -u tools/probes/svdpp_long_chain.py gpurun_out/${tag}_chain.jsonl > gpurun_out/${tag}_chain.log 2>&1; rc=$?; cat gpurun_out/${tag}_chain.jsonl; exit $rc
