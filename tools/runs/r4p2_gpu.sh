# final-tree profiles, part 2: C4 (SVD K=128 fp32) and the C5 shard (SVD++ K=128 fp32)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r4p}
DTYPE=f32 bash tools/profile.sh ${TAG}_c4 --shape c4 && \
DTYPE=f32 bash tools/profile.sh ${TAG}_c5 --shape c5 --users 1250000
