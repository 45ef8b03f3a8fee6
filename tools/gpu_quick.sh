# usage (on the GPU box): bash tools/gpu_quick.sh TAG [pytest -k expr] -- focused GPU parity tests, the
# default bench line (RMSE leg included, no CPU baseline / SVD++ leg) and a kernel trace of it
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-q}; K=${2:-"log or ckpt or split"}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-svdpp > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline --no-rmse --no-svdpp --steps 20 --warmup 3 > gpurun_out/prof_${TAG}_bench.log 2>&1 || exit $?
cut -d, -f1-4 gpurun_out/prof_$TAG/run_kernel_stats.csv | head -8
