#!/bin/bash
# round 5: two timing probes in one call -- r5r (the headline's log stores non-temporal per launch
# group) and r5s (what the item row's bias line costs the C4 gathers)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/runs/r5r_gpu.sh && bash tools/runs/r5s_gpu.sh
