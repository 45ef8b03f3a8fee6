#!/bin/bash
# round 5 final rehearsal, part 1 (the final tree): every GPU test outside test_gpu_scale.py, then
# smoke(), then the default bench line and the rocprofv3 kernel trace + stats of that command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${TAG:-r5f}
fatal() { case $1 in 124|137|134|139) echo "step rc $1: stopping"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests --ignore=tests/test_gpu_scale.py -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed" gpurun_out/${tag}_pytest.log | tail -4; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${tag}_smoke.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err; rc=$?; tail -1 gpurun_out/${tag}_bench.err; fatal $rc; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${tag}_default -o run -- python3 $GRAFT_REPO_ROOT/bench.py --detail $GRAFT_REPO_ROOT/gpurun_out/prof_${tag}_default_detail.json > $GRAFT_REPO_ROOT/gpurun_out/prof_${tag}_default_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_${tag}_default_bench.err; rc=$?
cd $GRAFT_REPO_ROOT; echo "rocprof rc $rc"; head -c 600 gpurun_out/${tag}_bench.json; echo; exit $rc
