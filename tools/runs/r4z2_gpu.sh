# final rehearsal, part 2: smoke() and the default bench line (driver order)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; TAG=${1:-r4z}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log
rc=$?; tail -2 gpurun_out/${TAG}_bench.log; grep '^{' gpurun_out/${TAG}_bench.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r['roofline']['frac'], r.get('rmse',{}).get('delta'), (r.get('c4') or {}).get('ms_per_step'))"; exit $rc
