# usage (on the GPU box): bash tools/gpu_full.sh TAG -- pytest -m gpu, smoke(), the default bench
# line (with cpu_baseline and rmse), then the rocprofv3 kernel-trace + PMC passes of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r}
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -rf > gpurun_out/${TAG}_pytest.log 2>&1
echo "pytest exit $?"; tail -5 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
bash tools/profile.sh ${TAG}
