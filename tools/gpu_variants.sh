# usage (on the GPU box): bash tools/gpu_variants.sh TAG MODE v1 v2 ... -- chain probe (fast cases)
# with the product library and each build_exp/lib_<v>.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=$1; MODE=$2; shift 2
echo "== product"; timeout -k 10 300 python tools/chain_probe.py $MODE 100 fast 2>&1 | grep -v amdgpu.ids || exit 1
for v in "$@"; do
  echo "== $v"
  SURPRISE_AMD_LIB=build_exp/lib_$v.so timeout -k 10 300 python tools/chain_probe.py $MODE 100 fast 2>&1 | grep -v amdgpu.ids || exit 1
done
