# usage (on the GPU box): [DTYPE=f32] bash tools/profile.sh TAG [extra bench args, e.g. --algo svdpp]
# 1) kernel trace + stats of the bench; 2) FETCH_SIZE and WRITE_SIZE in separate --pmc passes
#    (MI355X_MICROARCH.md HBM/rocprofv3: one TCC counter group per pass), 3) TCC hit / miss;
# then python3 tools/summarize_prof.py TAG (here, after the merge) writes profiles/TAG_* and
# profiles/traffic_<algo>_k<K>_<shape>.json (HBM bytes of one step summed over every kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r}
shift
EXTRA="$*"
mkdir -p gpurun_out
B="bench.py --no-cpu-baseline --no-rmse --no-svdpp --no-predict --no-chain-probe --no-c4 --dtype ${DTYPE:-f64}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 $B --steps 20 --warmup 3 $EXTRA --detail gpurun_out/prof_${TAG}_detail.json > gpurun_out/prof_${TAG}_bench.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pmc_fetch_$TAG -o run -- python3 $B --steps 5 --warmup 1 $EXTRA > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/pmc_write_$TAG -o run -- python3 $B --steps 5 --warmup 1 $EXTRA > gpurun_out/pmc_write_${TAG}.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d gpurun_out/pmc_l2_$TAG -o run -- python3 $B --steps 5 --warmup 1 $EXTRA > gpurun_out/pmc_l2_${TAG}.log 2>&1 || exit $?
echo "profile $TAG done"
