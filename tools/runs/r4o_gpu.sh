# three-group split with the rest of the heavy users on XCD 1 (the top chains alone on XCD 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -k "headline or native_fork" > gpurun_out/r4o_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; tail -2 gpurun_out/r4o_pytest.log; [ $rc -eq 0 ] || exit $rc
B="python3 -u bench.py --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 50 --warmup 5"
for v in "t16a:" "t0a:--top 0" "t32:--top 32" "t64:--top 64" "t16b:" "t0b:--top 0" "t16f32:--dtype f32" "t0f32:--dtype f32 --top 0"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 120 $B $args > gpurun_out/r4o_$name.json 2> gpurun_out/r4o_$name.log || exit $?
  grep '^{' gpurun_out/r4o_$name.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; ek=ph['epoch_kernel']; print('$name', r['dtype'], round(r['ms_per_step'],4), '%.3e' % r['value'], {k: round(v*1e3,1) for k, v in ph.items() if k.endswith('_ms')}, {k: round(v['avg_us'],1) for k, v in ek['launches'].items()})"
done
