#!/bin/bash
# round 5 GPU call: selected GPU tests (-k expression $2 over the files $3), then (unless $4=nobench)
# the default bench.  usage: tools/r5_gpu.sh TAG "K-EXPR" "FILES" [nobench]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=$1; kexpr=$2; files=${3:-tests}
if [ -n "$kexpr" ]; then
  timeout -k 10 780 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread $files \
      -m gpu -k "$kexpr" -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1 \
      || { tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
  grep -E "PASSED|FAILED|passed|failed|c5_u60000" gpurun_out/${tag}_pytest.log | tail -30
fi
if [ "$4" != "nobench" ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
  rc=$?
  tail -4 gpurun_out/${tag}_bench.err
  wc -c gpurun_out/${tag}_bench.json
  exit $rc
fi
