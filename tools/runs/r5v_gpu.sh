#!/bin/bash
# round 5: the SB epoch's item-bias mirror (ABI 934: mf_svd_epoch_sq item_bias, mf_log_apply
# bias_out, 128-B item rows) -- the parity file, the C4 scale tests (E=20 vs the committed
# oracle, fp32 and fp64), then C4 fp32 / fp64 timing with the mirror on and off, and the headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5v
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; ph=rl.get('phases_gpu_ms',{}); print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'epoch', ph.get('epoch_kernel_ms'), 'replay', ph.get('replay_ms'), 'fold', ph.get('fold_sync_ms'))"; }
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_abi.py -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed|k128_checkpoint" gpurun_out/${tag}_pytest.log | tail -12; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -v -s --timeout 800 --timeout-method thread -m gpu tests/test_gpu_scale.py -k "c4" -p no:cacheprovider > gpurun_out/${tag}_scale.log 2>&1; rc=$?; echo "scale rc $rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/${tag}_scale.log | tail -6; fatal $rc; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for m in 1 0; do
    for dt in f32 f64; do
      timeout -k 10 200 python3 -u bench.py --shape c4 --dtype $dt --bias-mirror $m --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 5 --warmup 2 --detail gpurun_out/${tag}_m${m}_${dt}_${rep}_d.json > gpurun_out/${tag}_m${m}_${dt}_${rep}.json 2> gpurun_out/${tag}_m${m}_${dt}_${rep}.log; rc=$?; show ${tag}_m${m}_${dt}_${rep}; fatal $rc
    done
  done
done
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err; rc=$?; tail -2 gpurun_out/${tag}_bench.err; head -c 1500 gpurun_out/${tag}_bench.json; echo; exit $rc
