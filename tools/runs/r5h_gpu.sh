#!/bin/bash
# round 5: r5e (the fused q-log fold: parity + the C5 shard timing + trace, the dispatch-check
# test) and r5g (log-store cache policy, id prefetch depth, light replay waves) in one call
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/runs/r5e_gpu.sh r5h || exit $?
bash tools/runs/r5g_gpu.sh r5h
