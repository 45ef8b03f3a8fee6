# usage (on the GPU box): bash tools/gpu_lib_env.sh VAR "v1 v2" lib1 lib2 ... -- short bench line per
# (library variant, env value); lib "product" = the in-tree library
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VAR=$1; VALS=$2; shift 2
show() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d["roofline"]; print("value %.3e ms/step %.4f epoch_ms %.4f rest_ms %.4f" % (d["value"], d["ms_per_step"], r["launch_ms"], r["rest_of_step_ms"]))'; }
for lib in "$@"; do for v in $VALS; do
  L=""; [ "$lib" != product ] && L="SURPRISE_AMD_LIB=build_exp/lib_$lib.so"
  echo -n "$lib $VAR=$v: "; env $L $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-rmse 2>/dev/null | show || exit 1
done; done
