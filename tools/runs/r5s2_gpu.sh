#!/bin/bash
# round 5: SVD++'s shared-step chain (s = p + m carried alone where lr_pu = lr_yj and reg_pu =
# reg_yj) -- every SVD++ GPU test of the parity / ext files and the C5-shard q-log E=20 scale test,
# then C3 (the bench's svdpp_c3 leg), the C5 shard on both schedules, and the one-chain probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5ss
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; ph=rl.get('phases_gpu_ms',{}); c3=r.get('svdpp_c3') or {}; print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'epoch', ph.get('epoch_kernel_ms'), 'fold', ph.get('fold_sync_ms'), 'c3', c3.get('ms_per_step'), (c3.get('f32_leg') or {}).get('ms_per_step'))"; }
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ext.py -k "svdpp or c3 or shared_step" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed" gpurun_out/${tag}_pytest.log | tail -6; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_scale.py -k "qlog_e20" -p no:cacheprovider > gpurun_out/${tag}_scale.log 2>&1; rc=$?; echo "scale rc $rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/${tag}_scale.log | tail -3; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-rmse --no-predict --no-c4 --no-chain-probe --steps 5 --warmup 2 --detail gpurun_out/${tag}_ml_d.json > gpurun_out/${tag}_ml.json 2> gpurun_out/${tag}_ml.log; rc=$?; show ${tag}_ml; fatal $rc
for q in 1 0; do
  timeout -k 10 300 python3 -u bench.py --shape c5 --users 1250000 --qlog $q --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1 --detail gpurun_out/${tag}_c5q${q}_d.json > gpurun_out/${tag}_c5q${q}.json 2> gpurun_out/${tag}_c5q${q}.log; rc=$?; show ${tag}_c5q${q}; fatal $rc
done
timeout -k 10 300 python3 -u tools/probes/svdpp_long_chain.py gpurun_out/${tag}_chain.jsonl > gpurun_out/${tag}_chain.log 2>&1; rc=$?; cat gpurun_out/${tag}_chain.jsonl | head -2; exit $rc
