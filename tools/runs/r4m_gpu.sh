# three-group heavy split (engine `top`): parity on the headline configuration and every split
# test, then the fp64 / fp32 headline with top = 16 (default), 8, 32 and 0 (the two-group split)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -k "headline or heavy or native_fork or blocked_solve or checkpoint or log_mode or n_ranks" > gpurun_out/r4m_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; tail -3 gpurun_out/r4m_pytest.log; [ $rc -eq 0 ] || exit $rc
B="python3 -u bench.py --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 50 --warmup 5"
for v in "t16a:" "t0a:--top 0" "t8:--top 8" "t32:--top 32" "t16b:" "t0b:--top 0" "t16f32:--dtype f32" "t0f32:--dtype f32 --top 0"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 120 $B $args > gpurun_out/r4m_$name.json 2> gpurun_out/r4m_$name.log || exit $?
  grep '^{' gpurun_out/r4m_$name.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; ek=ph['epoch_kernel']; print('$name', r['dtype'], round(r['ms_per_step'],4), '%.3e' % r['value'], {k: round(v*1e3,1) for k, v in ph.items() if k.endswith('_ms')}, {k: round(v['avg_us'],1) for k, v in ek['launches'].items()})"
done
