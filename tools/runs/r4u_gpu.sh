# after the bank change: the whole GPU suite, then the C4 profile (kernel stats + traffic)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; TAG=${1:-r4u}
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
DTYPE=f32 bash tools/profile.sh ${TAG}_c4 --shape c4
