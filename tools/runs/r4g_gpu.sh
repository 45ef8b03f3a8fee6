# The full C5 workload (10M users x 1M items x 1B ratings, SVD++ K=128 fp32) on ONE GPU: the N=1
# point of C5's strong-scaling curve, property-checked (held-out RMSE below the global mean's;
# no oracle runs at this size), chunks by the per-rank rule (125 at 10M users).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1100 python -u bench.py --shape c5 --steps 3 --warmup 1 --rmse-epochs 20 \
    --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe \
    > gpurun_out/r4g_c5full.json 2> gpurun_out/r4g_c5full.log || exit $?
grep '^{' gpurun_out/r4g_c5full.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], r['value'], r['rmse'])"
