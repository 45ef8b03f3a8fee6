#!/bin/bash
# round 5, first GPU call: the new configs[0] / forced-exchange tests, then the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${1:-r5a}
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_ext.py -k "configs0 or rccl or dispatch or headline_configuration or fp64_k128 or narrow" -p no:cacheprovider \
    > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -5 gpurun_out/${tag}_pytest.log
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
rc=$?
tail -3 gpurun_out/${tag}_bench.err
wc -c gpurun_out/${tag}_bench.json
exit $rc
