# usage (on the GPU box): bash tools/gpu_chain.sh TAG [MODE] -- pytest (parity file only) + SVD chain probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-c}; MODE=${2:-log}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/chain_probe.py $MODE > gpurun_out/${TAG}_chain.log 2>&1 && grep -v amdgpu.ids gpurun_out/${TAG}_chain.log
