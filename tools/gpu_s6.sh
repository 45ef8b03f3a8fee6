# usage (on the GPU box): bash tools/gpu_s6.sh -- pytest -m gpu, the SVD++ chain probe and bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s6_pytest.log 2>&1; echo "pytest exit $?"; tail -3 gpurun_out/s6_pytest.log
PROBE_ALGO=svdpp timeout -k 10 300 python tools/chain_probe.py atomic > gpurun_out/s6_chain_pp.log 2>&1 && grep -v amdgpu.ids gpurun_out/s6_chain_pp.log &&
timeout -k 10 300 python bench.py --algo svdpp --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/s6_bench_pp.log 2>&1 && tail -1 gpurun_out/s6_bench_pp.log
