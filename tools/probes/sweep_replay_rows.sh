# usage (GPU box): bash tools/sweep_replay_rows.sh -- SVD checkpoint log at ML-1M: light-group replay
# piece length (the fold sums fewer, longer pieces per item)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-rmse --no-svdpp --no-predict --steps 40 --warmup 5"
for dt in f32 f64; do for r in 64 128 256 512; do
  timeout -k 10 120 $B --dtype $dt --replay-rows $r > gpurun_out/rr_${dt}_$r.json 2>gpurun_out/rr_err.log || exit $?
  python -c "import json;d=json.load(open('gpurun_out/rr_${dt}_$r.json'));p=d['roofline']['phases_gpu_ms'];print('$dt replay rows $r', round(d['ms_per_step'],4), 'epoch', round(p['epoch_kernel_ms'],4), 'replay', round(p['replay_ms'],4), 'fold', round(p['fold_sync_ms'],4))"
done; done
