set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -k "blocked_solve or headline_configuration" > gpurun_out/r4c_pytest_gram.log 2>&1; rc=$?; echo "gram pytest rc $rc"; tail -3 gpurun_out/r4c_pytest_gram.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-c4 --steps 50 --warmup 5"
for v in "def:" "la:--gram 0" "gx:--gram 1 --xcd-split 1 --heavy 128" "g128:--gram 1 --heavy 128" "g512:--gram 1 --heavy 512" "la32:--gram 0 --dtype f32" "g32:--dtype f32"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 120 $B $args > gpurun_out/r4c_var_$name.json 2> gpurun_out/r4c_var_$name.log || { echo "variant $name failed"; exit 1; }
  python -c "import json,sys; r=json.loads([l for l in open('gpurun_out/r4c_var_$name.json') if l.startswith('{')][0]); print('$name', r['dtype'], round(r['ms_per_step'],4), '%.3e'%r['value'], r['roofline'].get('chain_latency',{}).get('alone_us'))"
done
timeout -k 10 800 python -u -m pytest tests -x -v -m gpu --timeout 700 --timeout-method thread -k "rccl or helper_ring or test_c3_ml1m or unbiased_k100 or tracks_multirank or c5_at_8_ranks or bench_two_ranks" > gpurun_out/r4c_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; tail -5 gpurun_out/r4c_pytest.log; exit $rc
