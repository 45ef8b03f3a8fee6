# usage (on the GPU box): bash tools/gpu_profiles.sh TAG -- rocprofv3 kernel stats + HBM traffic
# (FETCH_SIZE / WRITE_SIZE in separate --pmc passes) of every configuration the bench line
# reports: ML-1M SVD fp64 (the headline) and fp32, SVD++ C3 fp64 and fp32, C4 SVD fp32, and the
# C5 shard (SVD++ K=128 fp32, 1.25M users).
# Then, in the build container: for t in TAG_svd64 TAG_svd32 TAG_pp64 TAG_pp32 TAG_c4 TAG_c5; do
#   python tools/summarize_prof.py $t; done
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4p}
DTYPE=f64 bash tools/profile.sh ${TAG}_svd64 && \
DTYPE=f32 bash tools/profile.sh ${TAG}_svd32 && \
DTYPE=f64 bash tools/profile.sh ${TAG}_pp64 --algo svdpp && \
DTYPE=f32 bash tools/profile.sh ${TAG}_pp32 --algo svdpp && \
DTYPE=f32 bash tools/profile.sh ${TAG}_c4 --shape c4 && \
DTYPE=f32 bash tools/profile.sh ${TAG}_c5 --shape c5 --users 1250000
