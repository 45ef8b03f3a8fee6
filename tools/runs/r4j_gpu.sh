# q log with item-grouped rows: parity, then the C5 shard (q log vs atomic) and the full C5 (q log)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -k "qlog" > gpurun_out/r4j_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; tail -3 gpurun_out/r4j_pytest.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --shape c5 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe"
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; print('$1', r['config']['workload'][-70:], round(r['ms_per_step'],2), 'epoch', round(ph['epoch_kernel_ms'],2), 'replay', round(ph['replay_ms'],2), 'fold', round(ph['fold_sync_ms'],2), 'rmse', (r.get('rmse') or {}).get('delta'))"; }
timeout -k 10 300 $B --users 1250000 --steps 3 --warmup 1 --no-rmse --qlog > gpurun_out/r4j_shard_qlog.json 2> gpurun_out/r4j_shard_qlog.log || exit $?; show r4j_shard_qlog
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r4j_shard_qlog -o run -- python3 -u bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 2 --warmup 1 --qlog > gpurun_out/r4j_shard_qlog_prof.json 2> gpurun_out/r4j_shard_qlog_prof.log || exit $?
head -8 gpurun_out/prof_r4j_shard_qlog/run_kernel_stats.csv | cut -c1-120
timeout -k 10 500 $B --steps 2 --warmup 1 --no-rmse --qlog > gpurun_out/r4j_full_qlog.json 2> gpurun_out/r4j_full_qlog.log || exit $?; show r4j_full_qlog
