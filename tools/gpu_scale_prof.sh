# usage (on the GPU box): bash tools/gpu_scale_prof.sh TAG -- rocprofv3 kernel stats of the C4-shape
# scale run (no oracle)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-sc}
timeout -k 10 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/ks_$TAG -o run -- python3 tools/scale_run.py --shape c4 --factors 128 --epochs 4 --no-oracle > gpurun_out/ks_${TAG}.log 2>&1 || exit $?
tail -1 gpurun_out/ks_${TAG}.log
f=$(find gpurun_out/ks_$TAG -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:8]:
    print('%-40s calls %5s avg_ms %8.3f' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e6))
"
