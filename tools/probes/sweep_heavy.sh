set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-rmse --no-svdpp --no-predict --steps 40 --warmup 5"
for dt in f32 f64; do for h in 32 64 96 128 192; do
  timeout -k 10 120 $B --dtype $dt --heavy $h > gpurun_out/hv_${dt}_$h.json 2>gpurun_out/hv_err.log || exit $?
  python -c "import json;d=json.load(open('gpurun_out/hv_${dt}_$h.json'));p=d['roofline']['phases_gpu_ms'];e=p['epoch_launches']['ms_and_ratings'];print('$dt heavy $h', round(d['ms_per_step'],4), 'heavy/light epoch', e, 'replay', round(p['replay_ms'],4), 'fold', round(p['fold_sync_ms'],4))"
done; done
