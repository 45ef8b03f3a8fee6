#!/bin/bash
# round 5: the fused fold with its indices two items ahead (parity, C5-shard timing), policy
# probes (the q log's drift vs chunks at C3; the deterministic fit's cost on u1), the full C5 on
# the atomic schedule with its RMSE leg (the long-chain dealing as shipped), and the C4 fp64
# kernel + HBM-counter profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5k
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); rl=r['roofline']; print('$1', 'ms/step', r['ms_per_step'], 'frac', rl.get('frac'), 'tfrac', rl.get('traffic_frac'), rl.get('phases_gpu_ms'))"; }
timeout -k 10 400 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "qlog" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/${tag}_pytest.log | tail -12; fatal $rc; [ $rc -eq 0 ] || exit $rc
B5="python3 -u bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1 --qlog"
timeout -k 10 240 $B5 --detail gpurun_out/${tag}_c5q_d.json > gpurun_out/${tag}_c5q.json 2> gpurun_out/${tag}_c5q.log; rc=$?; show ${tag}_c5q; fatal $rc
timeout -k 10 900 python3 -u tools/probes/qlog_chunks_exact_speed.py gpurun_out/r5k_probe.jsonl > gpurun_out/r5k_probe.log 2>&1; rc=$?
echo "probe rc $rc"; cat gpurun_out/r5k_probe.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python3 -u bench.py --shape c5 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 2 --warmup 1 --detail gpurun_out/r5k_c5full_atomic_detail.json > gpurun_out/r5k_c5full_atomic.json 2> gpurun_out/r5k_c5full_atomic.log; rc=$?
tail -2 gpurun_out/r5k_c5full_atomic.log; head -c 600 gpurun_out/r5k_c5full_atomic.json; echo
[ $rc -eq 0 ] || exit $rc
DTYPE=f64 bash tools/profile.sh r5k_c4_64 --shape c4
