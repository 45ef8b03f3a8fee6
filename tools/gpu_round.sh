# usage: bash tools/gpu_round.sh TAG   (runs on the GPU box; every GPU step has its own limit)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r}
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -rf --durations=10 > gpurun_out/${TAG}_pytest.log 2>&1
echo "pytest exit $?"; tail -30 gpurun_out/${TAG}_pytest.log
timeout -k 10 900 python tools/exp_modes.py all > gpurun_out/${TAG}_exp.log 2>&1
echo "exp exit $?"; head -2 gpurun_out/${TAG}_exp.log
for m in log atomic plain; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 3 --mode $m --no-cpu-baseline --no-rmse > gpurun_out/${TAG}_bench_$m.log 2>&1 || exit $?
  echo "$m $(tail -1 gpurun_out/${TAG}_bench_$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["launch_ms"], d["roofline"]["frac"])')"
done
