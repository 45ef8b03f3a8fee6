#!/bin/bash
# round 5: kernel breakdown of C3 (SVD++ K=100 fp32, the bench's svdpp_c3 leg) with the hybrid
# launch off / on (cold share 0.5): rocprofv3 kernel trace + stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cs in 0 0.5; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r5mp_cs$cs -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cold-share $cs --no-cpu-baseline --no-rmse --no-predict --no-c4 --no-chain-probe --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r5mp_cs$cs.json 2> $GRAFT_REPO_ROOT/gpurun_out/r5mp_cs$cs.log || exit $?
  cd $GRAFT_REPO_ROOT; echo "== cs $cs"; head -12 gpurun_out/prof_r5mp_cs$cs/run_kernel_stats.csv | cut -c1-160
done
