# usage (on the GPU box): bash tools/gpu_probe.sh TAG "<bench args>" [ENV=V[,ENV2=V2] ...]
# one bench line per env setting ("-" = none): ms/step and the per-phase GPU times, no profiler
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=$1; ARGS=$2; shift 2
for e in "$@"; do
  E=""; [ "$e" != "-" ] && E=$(echo "$e" | tr ',' ' ')
  env $E timeout -k 10 180 python bench.py --no-cpu-baseline --no-rmse --no-svdpp $ARGS > gpurun_out/${TAG}_probe.json 2> gpurun_out/${TAG}_probe.err || { tail -5 gpurun_out/${TAG}_probe.err; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/${TAG}_probe.json') if l.startswith('{')][-1])
ph=d['roofline']['phases_gpu_ms']
print('%-60s ms/step %.4f  epoch %.4f  replay/fold %.4f  sync %.4f  frac %.3f' % ('$e', d['ms_per_step'], ph.get('epoch_kernel_ms',0), ph.get('replay_ms',0), ph.get('fold_sync_ms',0), d['roofline']['frac']))"
done
