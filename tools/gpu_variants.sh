# usage (on the GPU box): bash tools/gpu_variants.sh TAG "<bench args>" NAME=ENV[,ENV2] ... -- a kernel trace per
# setting ("-" = none; ENV may be SURPRISE_AMD_LIB=surprise_amd/variants/libsurprise_amd_X.so): ms/step,
# then the per-kernel average durations of the trace (gpurun_out/pv_TAG_NAME)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
for spec in "$@"; do
  name=${spec%%=*}; e=${spec#*=}; E=""; [ "$e" != "-" ] && E=$(echo "$e" | tr ',' ' ')
  env $E timeout -k 10 180 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/pv_${TAG}_$name -o run -- python3 bench.py --no-cpu-baseline --no-rmse --no-svdpp --steps 12 --warmup 2 $ARGS > gpurun_out/pv_${TAG}_$name.log 2>&1 || { tail -5 gpurun_out/pv_${TAG}_$name.log; exit 1; }
  echo "== $name ($e): ms/step $(cat gpurun_out/pv_${TAG}_$name.log | python3 -c 'import json,sys; print(round(json.loads([l for l in sys.stdin if l.startswith("{")][-1])["ms_per_step"],4))')"
  python3 tools/timeline.py gpurun_out/pv_${TAG}_$name ${TL_N:-5}
done
