# usage (on the GPU box): bash tools/gpu_scale_ab.sh v1 ... -- C4-shape epochs (no oracle) with the
# product library and each build_exp/lib_<v>.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in product "$@"; do L=""; [ $lib != product ] && L="SURPRISE_AMD_LIB=build_exp/lib_$lib.so"
  echo -n "$lib: "; env $L timeout -k 10 600 python tools/scale_run.py --shape c4 --factors 128 --epochs 4 --no-oracle 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(["%.2f" % x for x in d["epoch_ms"]], "%.3e" % d["updates_per_s"])' || exit 1
done
