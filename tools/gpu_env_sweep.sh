# usage (on the GPU box): bash tools/gpu_env_sweep.sh VAR v1 v2 ... -- short bench line per value
# of the environment variable VAR
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VAR=$1; shift
show() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d["roofline"]; print("value %.3e ms/step %.4f epoch_ms %.4f rest_ms %.4f" % (d["value"], d["ms_per_step"], r["launch_ms"], r["rest_of_step_ms"]))'; }
for v in "$@"; do
  echo -n "$VAR=$v: "; env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-rmse 2>/dev/null | show || exit 1
done
