# usage (on the GPU box): bash tools/gpu_kstats.sh TAG [v] -- rocprofv3 kernel stats of a short
# bench (product library, or build_exp/lib_<v>.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=$1; V=$2
[ -n "$V" ] && export SURPRISE_AMD_LIB=build_exp/lib_$V.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/ks_$TAG -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-rmse > gpurun_out/ks_${TAG}.log 2>&1 || exit $?
f=$(find gpurun_out/ks_$TAG -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:12]:
    print('%-60s calls %6s avg_us %8.2f total_ms %8.3f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
"
