# usage (GPU box): bash tools/sweep_variants.sh NAME... -- the ML-1M SVD bench (fp64, fp32) with the
# in-tree library and with each experiment variant surprise_amd/variants/libsurprise_amd_NAME.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-rmse --no-svdpp --no-predict --steps 40 --warmup 5"
for v in base "$@"; do for dt in f64 f32; do
  if [ "$v" = base ]; then L=""; else L="surprise_amd/variants/libsurprise_amd_$v.so"; fi
  SURPRISE_AMD_LIB=$L timeout -k 10 120 $B --dtype $dt > gpurun_out/var_${v}_$dt.json 2>gpurun_out/var_err.log || exit $?
  python -c "import json;d=json.load(open('gpurun_out/var_${v}_$dt.json'));p=d['roofline']['phases_gpu_ms'];e=p['epoch_launches']['ms_and_ratings'];print('$v $dt', round(d['ms_per_step'],4), 'heavy/light epoch', e, 'replay', round(p['replay_ms'],4), 'fold', round(p['fold_sync_ms'],4))"
done; done
