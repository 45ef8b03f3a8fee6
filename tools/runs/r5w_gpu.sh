#!/bin/bash
# round 5: the item-bias mirror read by vector loads (r5v's scalar loads waited on the next
# bank's) -- the SB parity tests, then C4 fp32 / fp64 with the mirror on and off, two passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5w
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; ph=rl.get('phases_gpu_ms',{}); print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'epoch', ph.get('epoch_kernel_ms'), 'replay', ph.get('replay_ms'), 'fold', ph.get('fold_sync_ms'))"; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "k128_checkpoint or narrow or nontemporal or staggered or long_replay" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed" gpurun_out/${tag}_pytest.log | tail -6; fatal $rc; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for m in 1 0; do
    for dt in f32 f64; do
      timeout -k 10 200 python3 -u bench.py --shape c4 --dtype $dt --bias-mirror $m --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 5 --warmup 2 --detail gpurun_out/${tag}_m${m}_${dt}_${rep}_d.json > gpurun_out/${tag}_m${m}_${dt}_${rep}.json 2> gpurun_out/${tag}_m${m}_${dt}_${rep}.log; rc=$?; show ${tag}_m${m}_${dt}_${rep}; fatal $rc
    done
  done
done
