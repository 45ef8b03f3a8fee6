# usage (GPU box): bash tools/sweep_hx.sh [c5] -- SVD++ helper-wave launch: helpers per chain x
# chains per CU, C3 (ML-1M shape, fp32 + fp64) or the C5 per-rank shard
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ "$1" = "c5" ]; then
  B="python bench.py --shape c5 --users 1250000 --no-cpu-baseline --no-rmse --steps 3 --warmup 1"
  CASES="3:2 1:4"; DTS="f32"
else
  B="python bench.py --algo svdpp --no-cpu-baseline --no-rmse --no-svdpp --no-predict --steps 20 --warmup 3"
  CASES="3:2 1:2 1:3 1:4"; DTS="f32 f64"
fi
for dt in $DTS; do for c in $CASES; do h=${c%:*}; n=${c#*:}
  timeout -k 10 600 $B --dtype $dt --hx-helpers $h --hx-chains $n > gpurun_out/hx_${1}_${dt}_${h}_${n}.json 2>gpurun_out/hx_err.log || exit $?
  python -c "import json;d=json.load(open('gpurun_out/hx_${1}_${dt}_${h}_${n}.json'));p=d['roofline']['phases_gpu_ms'];print('$dt helpers $h chains/CU $n', round(d['ms_per_step'],4), 'ms/step, epoch kernel', round(p['epoch_kernel_ms'],4), 'fold', round(p['replay_ms'],4))"
done; done
