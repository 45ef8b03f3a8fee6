set -o pipefail
cd "$GRAFT_REPO_ROOT"
show() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d["roofline"]; print("value %.3e ms/step %.4f epoch_ms %.4f rest_ms %.4f" % (d["value"], d["ms_per_step"], r["launch_ms"], r["rest_of_step_ms"]))'; }
for lib in product u4; do L=""; [ $lib != product ] && L="SURPRISE_AMD_LIB=build_exp/lib_$lib.so"
echo -n "$lib K=128: "; env $L timeout -k 10 300 python bench.py --factors 128 --no-cpu-baseline --no-rmse 2>/dev/null | show || exit 1
done
