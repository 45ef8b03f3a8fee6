#!/bin/bash
# round 5 combined call: GPU tests of the new paths, then C5-shard q log (fused fold) vs atomic,
# C4 with / without the staggered halves (fp32 and fp64), then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r5d}
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -v -s --timeout 500 --timeout-method thread -m gpu \
  tests/test_gpu_dist.py tests/test_gpu_ext.py tests/test_gpu_scale.py tests/test_gpu_parity.py \
  -k "rccl or dispatch or miniature or c4_fp64 or qlog or stagger" -p no:cacheprovider \
  > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"
grep -E "PASSED|FAILED|passed|failed|c5_u60000" gpurun_out/${tag}_pytest.log | tail -40; fatal $rc
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline'].get('phases_gpu_ms',{}); print('$1', r['config']['workload'][-50:], 'ms/step', round(r['ms_per_step'],3), 'frac', r['roofline'].get('frac'), ph)"; }
B5="python3 -u bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1"
timeout -k 10 240 $B5 --qlog --detail gpurun_out/${tag}_c5q_detail.json > gpurun_out/${tag}_c5q.json 2> gpurun_out/${tag}_c5q.log; rc=$?; show ${tag}_c5q; fatal $rc
timeout -k 10 240 $B5 --detail gpurun_out/${tag}_c5a_detail.json > gpurun_out/${tag}_c5a.json 2> gpurun_out/${tag}_c5a.log; rc=$?; show ${tag}_c5a; fatal $rc
B4="python3 -u bench.py --shape c4 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 5 --warmup 2"
for st in 1 0; do for dt in f32 f64; do
  timeout -k 10 240 $B4 --stagger $st --dtype $dt --detail gpurun_out/${tag}_c4_s${st}_${dt}_detail.json > gpurun_out/${tag}_c4_s${st}_${dt}.json 2> gpurun_out/${tag}_c4_s${st}_${dt}.log; rc=$?; show ${tag}_c4_s${st}_${dt}; fatal $rc
done; done
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err; rc=$?
tail -4 gpurun_out/${tag}_bench.err; wc -c gpurun_out/${tag}_bench.json; exit $rc
