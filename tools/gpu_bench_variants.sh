# usage (on the GPU box): bash tools/gpu_bench_variants.sh v1 v2 ... -- short bench line (no CPU
# baseline / RMSE; extra bench args in $BENCH_ARGS) with the product library and each build_exp/lib_<v>.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
show() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d["roofline"]; print("value %.3e ms/step %.4f kernel_ms %.4f merge_ms %.4f" % (d["value"], d["ms_per_step"], r["launch_ms"], r["rest_of_step_ms"]))'; }
echo -n "product: "; timeout -k 10 300 python bench.py --no-cpu-baseline --no-rmse $BENCH_ARGS 2>/dev/null | show || exit 1
for v in "$@"; do
  echo -n "$v: "; SURPRISE_AMD_LIB=build_exp/lib_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-rmse $BENCH_ARGS 2>/dev/null | show || exit 1
done
