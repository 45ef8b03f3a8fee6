# usage (on the GPU box): bash tools/gpu_svdpp_prof.sh TAG -- rocprofv3 summary of the SVD++ bench
# (deferred y fold) and the one-rank share of configs[4] (c5-shard, SVD++ K=128)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; TAG=${1:-r1_svdpp_ydefer}
bash tools/profile.sh $TAG --algo svdpp || exit $?
timeout -k 10 600 python3 -u tools/scale_run.py --shape c5-shard --algo svdpp --factors 128 --epochs 3 --no-oracle > gpurun_out/${TAG}_c5.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_c5.log; exit $rc
