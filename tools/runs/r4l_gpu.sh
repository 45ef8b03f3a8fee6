# y fold with single-piece items applied by their piece's wave: SVD++ parity, then the C5 shard
# (atomic default) and the full C5
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "svdpp or y_fold or c3_ml1m" > gpurun_out/r4l_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; tail -3 gpurun_out/r4l_pytest.log; [ $rc -eq 0 ] || exit $rc
B="python3 -u bench.py --shape c5 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse"
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; print('$1', r['config']['workload'][-70:], round(r['ms_per_step'],2), {k: round(v,2) for k, v in ph.items() if isinstance(v, float)})"; }
timeout -k 10 300 $B --users 1250000 --steps 3 --warmup 1 > gpurun_out/r4l_shard.json 2> gpurun_out/r4l_shard.log || exit $?; show r4l_shard
timeout -k 10 500 $B --steps 2 --warmup 1 > gpurun_out/r4l_full.json 2> gpurun_out/r4l_full.log || exit $?; show r4l_full
# replay piece length at the headline (fp64 ML-1M): the fold sums fewer pieces with longer ones
for rr in 64 128 256; do
  timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 50 --warmup 5 --replay-rows $rr > gpurun_out/r4l_rr$rr.json 2> gpurun_out/r4l_rr$rr.log || exit $?
  grep '^{' gpurun_out/r4l_rr$rr.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; print('rr $rr', round(r['ms_per_step'],4), {k: round(v*1e3,1) for k, v in ph.items() if k.endswith('_ms')})"
done
