# usage (on the GPU box): bash tools/gpu_dist.sh TAG -- the 2-rank GPU tests and a 2-rank bench
# rehearsal (two processes on the box's one GPU, gloo collectives)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; TAG=${1:-d}
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --backend gloo > gpurun_out/${TAG}_bench2.log 2>&1; rc=$?
echo "bench2 exit $rc"; grep '^{' gpurun_out/${TAG}_bench2.log | cut -c1-400
