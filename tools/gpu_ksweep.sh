# usage (on the GPU box): bash tools/gpu_ksweep.sh MODE K1 K2 ... -- chain probe (fast cases) per n_factors
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
MODE=$1; shift
for k in "$@"; do
  echo "== K=$k"; timeout -k 10 300 python tools/chain_probe.py $MODE $k fast 2>&1 | grep -v amdgpu.ids || exit 1
done
