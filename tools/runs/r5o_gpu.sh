#!/bin/bash
# round 5: cache policy of the epoch kernel's streams: snt = CSR reads + user rows non-temporal,
# snte = also the error-log stores (MF_STREAM_AUX, MF_ELOG_AUX) vs the product; C4 fp32 / fp64, headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5o
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; ph=rl.get('phases_gpu_ms',{}); print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'epoch', ph.get('epoch_kernel_ms'), 'replay', ph.get('replay_ms'), 'fold', ph.get('fold_sync_ms'))"; }
for v in base snt snte base snt snte; do
  lib=""; [ $v != base ] && lib="SURPRISE_AMD_LIB=tests/variants/libsurprise_amd_$v.so"
  for dt in f32 f64; do
    env $lib timeout -k 10 200 python3 -u bench.py --shape c4 --dtype $dt --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 5 --warmup 2 --detail gpurun_out/${tag}_${v}_c4${dt}_d.json > gpurun_out/${tag}_${v}_c4${dt}.json 2> gpurun_out/${tag}_${v}_c4${dt}.log; rc=$?; show ${tag}_${v}_c4${dt}; fatal $rc
  done
  env $lib timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --steps 30 --warmup 5 --detail gpurun_out/${tag}_${v}_ml_d.json > gpurun_out/${tag}_${v}_ml.json 2> gpurun_out/${tag}_${v}_ml.log; rc=$?; show ${tag}_${v}_ml; fatal $rc
done
