# final-tree profiles, part 1: ML-1M SVD fp64 / fp32, SVD++ C3 fp64 / fp32 (tools/profile.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r4p}
DTYPE=f64 bash tools/profile.sh ${TAG}_svd64 && \
DTYPE=f32 bash tools/profile.sh ${TAG}_svd32 && \
DTYPE=f64 bash tools/profile.sh ${TAG}_pp64 --algo svdpp && \
DTYPE=f32 bash tools/profile.sh ${TAG}_pp32 --algo svdpp
