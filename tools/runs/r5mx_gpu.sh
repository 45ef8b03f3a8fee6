#!/bin/bash
# round 5: the hybrid SVD++ launch (mf_svdpp_epoch_mix: cold items' gradients to an item-grouped
# log, the rest on the helper waves' float atomics) -- parity (all-cold vs the stalelog oracle,
# RMSE with half the ratings cold, the SVD++ atomic tests), then C3 timing at cold shares 0 / 0.3
# / 0.5 / 0.7 (the bench's svdpp_c3 leg) with its E=20 RMSE vs the exact oracle
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r5mx
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ext.py -k "hybrid or svdpp_parallel or svdpp_atomic or hot_row or item_bias or helper_ring or shared_step" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/${tag}_pytest.log | tail -8; fatal $rc; [ $rc -eq 0 ] || exit $rc
for cs in 0 0.3 0.5 0.7; do
  timeout -k 10 300 python3 -u bench.py --cold-share $cs --no-cpu-baseline --no-rmse --no-predict --no-c4 --no-chain-probe --steps 5 --warmup 2 --detail gpurun_out/${tag}_cs${cs}_d.json > gpurun_out/${tag}_cs${cs}.json 2> gpurun_out/${tag}_cs${cs}.log; rc=$?
  python -c "import json; r=json.load(open('gpurun_out/${tag}_cs${cs}_d.json')); c=r['svdpp_c3']; print('cold_share $cs', 'c3 f64', round(c['ms_per_step'],4), 'f32', round(c['f32_leg']['ms_per_step'],4))"; fatal $rc
done
timeout -k 10 400 python3 -u tools/probes/svdpp_c3_rmse.py gpurun_out/${tag}_rmse.jsonl > gpurun_out/${tag}_rmse.log 2>&1; rc=$?; cat gpurun_out/${tag}_rmse.jsonl; exit $rc
