# final rehearsal, part 1: the whole GPU suite as the driver runs it
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; TAG=${1:-r4z}
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_pytest.log; exit $rc
