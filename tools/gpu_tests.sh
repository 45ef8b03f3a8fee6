set -o pipefail
cd "$GRAFT_REPO_ROOT"
nproc; rocm-smi --showproductname 2>&1 | head -20 || true
timeout -k 10 1200 python -m pytest tests/test_gpu_parity.py -q -m gpu -rf --durations=15 > gpurun_out/r1_pytest.log 2>&1
echo "pytest exit $?"
tail -40 gpurun_out/r1_pytest.log
