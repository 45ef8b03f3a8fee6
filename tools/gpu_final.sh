# usage (on the GPU box): bash tools/gpu_final.sh TAG -- what the driver runs at round end:
# pytest -m gpu, smoke(), the default bench line (with CPU baseline and RMSE), in that order
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; TAG=${1:-f}
timeout -k 10 1200 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_bench.log; exit $rc
