#!/bin/bash
# round 5: cache policy of the epoch kernels' checkpoint-log stores (MF_LOG_AUX: 0 default,
# 16 = sc1 -- the line leaves the XCD's L2, 2 = nt) on the headline (ML-1M fp64 + fp32 leg) and C4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r5g}
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'span', rl.get('dominant_kernel',{}).get('span_us_per_step'), 'f32', (r.get('f32_leg') or {}).get('ms_per_step'), {k:v.get('avg_us') for k,v in rl.get('dominant_kernel',{}).get('launches',{}).items()})"; }
for w in 4 8; do
  timeout -k 10 200 python3 -u bench.py --light-replay-wpc $w --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --steps 30 --warmup 5 --detail gpurun_out/${tag}_lrw${w}_d.json > gpurun_out/${tag}_lrw${w}.json 2> gpurun_out/${tag}_lrw${w}.log; rc=$?; show ${tag}_lrw${w}; fatal $rc
done
for v in base aux16 aux2 ids3 ids4 ids8; do
  lib=""; [ $v != base ] && lib="SURPRISE_AMD_LIB=tests/variants/libsurprise_amd_$v.so"
  for rep in 1 2; do
    env $lib timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --steps 30 --warmup 5 --detail gpurun_out/${tag}_${v}_${rep}_d.json > gpurun_out/${tag}_${v}_${rep}.json 2> gpurun_out/${tag}_${v}_${rep}.log; rc=$?; show ${tag}_${v}_${rep}; fatal $rc
  done
  for dt in f32 f64; do
    env $lib timeout -k 10 200 python3 -u bench.py --shape c4 --dtype $dt --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 5 --warmup 2 --detail gpurun_out/${tag}_${v}_c4${dt}_d.json > gpurun_out/${tag}_${v}_c4${dt}.json 2> gpurun_out/${tag}_${v}_c4${dt}.log; rc=$?; show ${tag}_${v}_c4${dt}; fatal $rc
  done
done
