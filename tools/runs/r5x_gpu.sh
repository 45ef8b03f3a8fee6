#!/bin/bash
# round 5: HBM-counter profiles on the current tree -- the headline (fp64), C4 fp32 and C4 fp64
# (tools/profile.sh: kernel trace + stats, FETCH_SIZE / WRITE_SIZE / TCC hit passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
DTYPE=f64 bash tools/profile.sh r5x_ml64 && DTYPE=f32 bash tools/profile.sh r5x_c4_32 --shape c4 && DTYPE=f64 bash tools/profile.sh r5x_c4_64 --shape c4
