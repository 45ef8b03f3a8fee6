# usage (on the GPU box): bash tools/gpu_nmf_prof.sh TAG -- rocprofv3 kernel stats of the NMF /
# baseline-ALS timing run (tools/bench_ext.py), top kernels printed
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out; TAG=${1:-nmf}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/ks_$TAG -o run -- python3 tools/bench_ext.py > gpurun_out/ks_${TAG}.log 2>&1 || exit $?
f=$(find gpurun_out/ks_$TAG -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:8]:
    print('%-40s calls %5s avg_us %8.2f' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))
"
