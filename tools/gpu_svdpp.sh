# usage (on the GPU box): bash tools/gpu_svdpp.sh TAG -- pytest -m gpu, then the SVD++ bench line
# with the deferred y fold (default) and with the end-of-user atomics (SURPRISE_AMD_YDEFER=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; TAG=${1:-p}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
show() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d["roofline"]; print("value %.3e ms/step %.4f epoch_ms %.4f rest_ms %.4f" % (d["value"], d["ms_per_step"], r["launch_ms"], r["rest_of_step_ms"]))'; }
for v in 1 0; do echo -n "YDEFER=$v: "; SURPRISE_AMD_YDEFER=$v timeout -k 10 300 python bench.py --algo svdpp --no-cpu-baseline 2>/dev/null | show || exit 1; done
