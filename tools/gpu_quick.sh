# usage (on the GPU box): bash tools/gpu_quick.sh TAG -- pytest -m gpu, the SVD chain probe and
# the default bench line; every GPU step under its own time limit, stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/chain_probe.py log > gpurun_out/${TAG}_chain.log 2>&1 && grep -v amdgpu.ids gpurun_out/${TAG}_chain.log &&
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 && tail -1 gpurun_out/${TAG}_bench.log
