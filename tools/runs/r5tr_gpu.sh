#!/bin/bash
# round 5 final-tree traffic files (tags r5h_*; run as tools/runs/r5tr_gpu.sh): ML-1M SVD fp32, SVD++ C3 fp32 / fp64 (tools/profile.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
DTYPE=f32 bash tools/profile.sh r5h_ml32 && \
DTYPE=f32 bash tools/profile.sh r5h_pp32 --algo svdpp && \
DTYPE=f64 bash tools/profile.sh r5h_pp64 --algo svdpp
