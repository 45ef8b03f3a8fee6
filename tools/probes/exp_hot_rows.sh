# GPU-box experiment: SVD++ hot-row replica counts at C3 (ML-1M shape, K=100) and the C5 shard
# (auto policy vs none), after the SVD++ parity tests.  usage: bash tools/exp_hot_rows.sh
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --algo svdpp --dtype f32 --no-cpu-baseline --no-predict --no-svdpp --no-rmse --steps 30"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "svdpp or narrow" > gpurun_out/pp.log 2>&1 || exit 1
tail -1 gpurun_out/pp.log
for h in -1 0 2 4 8 16 32; do
  timeout -k 10 120 $B --hot-rows $h > gpurun_out/h_$h.log 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/h_$h.log').read().strip().splitlines()[-1]); print('hot $h', d['ms_per_step'], d['roofline']['phases_gpu_ms']['epoch_kernel_ms'])"
done
for h in -1 0; do
  timeout -k 10 300 python -u bench.py --shape c5 --users 1250000 --steps 3 --warmup 1 --no-rmse --no-cpu-baseline --no-predict --hot-rows $h > gpurun_out/c5_$h.log 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/c5_$h.log').read().strip().splitlines()[-1]); print('c5 hot $h', d['ms_per_step'], d['roofline']['phases_gpu_ms']['epoch_kernel_ms'])"
done
