set -o pipefail
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
echo -n "events: "; timeout -k 10 300 python bench.py --no-cpu-baseline --no-rmse --steps 50 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"])' || exit 1
echo -n "no events: "; BENCH_NO_EVENTS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-rmse --steps 50 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"])' || exit 1
done
