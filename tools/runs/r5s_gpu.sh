#!/bin/bash
# round 5: what the item row's bias line costs the C4 epoch kernel's gathers (timing probe):
# item rows padded to 64 B (the product) or 128 B (factor columns on whole lines), with the SB
# body's bias load (base) or without it (nb: MF_SB_NO_BIAS_LOAD, wrong numbers, timing only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5s
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; ph=rl.get('phases_gpu_ms',{}); print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'epoch', ph.get('epoch_kernel_ms'), 'replay', ph.get('replay_ms'), 'fold', ph.get('fold_sync_ms'))"; }
for rep in 1 2; do
  for v in base:64 base:128 nb:128; do
    lib=${v%%:*}; al=${v##*:}
    env=""; [ $lib != base ] && env="SURPRISE_AMD_LIB=tests/variants/libsurprise_amd_$lib.so"
    for dt in f32 f64; do
      env $env timeout -k 10 200 python3 -u bench.py --shape c4 --dtype $dt --item-align $al --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 5 --warmup 2 --detail gpurun_out/${tag}_${lib}${al}_${dt}_${rep}_d.json > gpurun_out/${tag}_${lib}${al}_${dt}_${rep}.json 2> gpurun_out/${tag}_${lib}${al}_${dt}_${rep}.log; rc=$?; show ${tag}_${lib}${al}_${dt}_${rep}; fatal $rc
    done
  done
done
