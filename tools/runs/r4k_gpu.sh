# q log with user_sq and the two-piece log reduce: parity (q log + every log-mode test), then the
# C5 shard q log vs atomic with a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -k "qlog or log_mode or gradient_log or svdpp_tracks_multirank or n_ranks" > gpurun_out/r4k_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; tail -3 gpurun_out/r4k_pytest.log; [ $rc -eq 0 ] || exit $rc
B="python3 -u bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --no-rmse --steps 3 --warmup 1"
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; print('$1', r['config']['workload'][-70:], round(r['ms_per_step'],2), {k: round(v,2) for k, v in ph.items() if isinstance(v, float)})"; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r4k_qlog -o run -- $B --qlog > gpurun_out/r4k_qlog.json 2> gpurun_out/r4k_qlog.log || exit $?; show r4k_qlog
head -9 gpurun_out/prof_r4k_qlog/run_kernel_stats.csv | cut -c1-110
