#!/bin/bash
# round 5: non-temporal log stores (MF_EPOCH_LOG_NT) -- parity, C4 fp32 / fp64 (auto: on), the
# C5 shard q log with and without them, then the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r5i}
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "nontemporal or qlog or headline_configuration" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/${tag}_pytest.log | tail -16; fatal $rc
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'tfrac', rl.get('traffic_frac'), rl.get('phases_gpu_ms'))"; }
B4="python3 -u bench.py --shape c4 --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 5 --warmup 2"
for dt in f32 f64; do
  timeout -k 10 200 $B4 --dtype $dt --detail gpurun_out/${tag}_c4${dt}_d.json > gpurun_out/${tag}_c4${dt}.json 2> gpurun_out/${tag}_c4${dt}.log; rc=$?; show ${tag}_c4${dt}; fatal $rc
done
B5="python3 -u bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1 --qlog"
for nt in 1 0; do
  timeout -k 10 240 $B5 --log-nt $nt --detail gpurun_out/${tag}_c5q${nt}_d.json > gpurun_out/${tag}_c5q${nt}.json 2> gpurun_out/${tag}_c5q${nt}.log; rc=$?; show ${tag}_c5q${nt}; fatal $rc
done
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err; rc=$?
tail -4 gpurun_out/${tag}_bench.err; cat gpurun_out/${tag}_bench.json | head -c 4000; exit $rc
