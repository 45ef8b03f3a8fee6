# q log (SVD++ without float atomics): parity tests, then the C5 shard and the full C5 with and
# without it (full C5: the long-chain users grouped into chunk 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "qlog or item_bias_beside or svdpp_parallel_rmse or c3_ml1m" > gpurun_out/r4i_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; tail -4 gpurun_out/r4i_pytest.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --shape c5 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe"
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; print('$1', r['config']['workload'][-70:], round(r['ms_per_step'],2), 'epoch', round(ph['epoch_kernel_ms'],2), 'replay', round(ph['replay_ms'],2), 'fold', round(ph['fold_sync_ms'],2), 'rmse', r.get('rmse'))"; }
timeout -k 10 400 $B --users 1250000 --steps 3 --warmup 1 --rmse-epochs 20 --qlog > gpurun_out/r4i_shard_qlog.json 2> gpurun_out/r4i_shard_qlog.log || exit $?; show r4i_shard_qlog
timeout -k 10 300 $B --users 1250000 --steps 3 --warmup 1 --no-rmse > gpurun_out/r4i_shard_atomic.json 2> gpurun_out/r4i_shard_atomic.log || exit $?; show r4i_shard_atomic
timeout -k 10 500 $B --steps 2 --warmup 1 --no-rmse > gpurun_out/r4i_full_atomic.json 2> gpurun_out/r4i_full_atomic.log || exit $?; show r4i_full_atomic
timeout -k 10 500 $B --steps 2 --warmup 1 --no-rmse --qlog > gpurun_out/r4i_full_qlog.json 2> gpurun_out/r4i_full_qlog.log || exit $?; show r4i_full_qlog
