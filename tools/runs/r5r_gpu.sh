#!/bin/bash
# round 5: the headline's checkpoint-log stores non-temporal per launch group (engine log_nt
# "heavy" / "light") vs none / both, two passes each (the replay's row gathers are nt already)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5r
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; ph=rl.get('phases_gpu_ms',{}); L=rl.get('dominant_kernel',{}).get('launches',{}); print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'epoch', ph.get('epoch_kernel_ms'), 'replay', ph.get('replay_ms'), 'fold', ph.get('fold_sync_ms'), {k: v.get('avg_us') for k, v in L.items()})"; }
for rep in 1 2; do
  for v in 0 heavy light 1; do
    timeout -k 10 200 python3 -u bench.py --log-nt $v --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --steps 30 --warmup 5 --detail gpurun_out/${tag}_${v}_${rep}_d.json > gpurun_out/${tag}_${v}_${rep}.json 2> gpurun_out/${tag}_${v}_${rep}.log; rc=$?; show ${tag}_${v}_${rep}; fatal $rc
  done
done
