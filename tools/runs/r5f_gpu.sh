#!/bin/bash
# round 5: (1) the fp64 C4 profile (kernel trace + FETCH_SIZE / WRITE_SIZE / L2 passes: the
# c4_f64 leg's traffic file), (2) the full C5 on one GPU (10M users, 990M training ratings,
# SVD++ K=128 fp32) on the final dealing with its 20-epoch RMSE leg, with the
# atomic schedule and with the q log (fused fold, nt log stores)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
DTYPE=f64 bash tools/profile.sh r5f_c4_64 --shape c4 || exit $?
for m in atomic qlog; do
  x=""; [ $m = qlog ] && x="--qlog"
  timeout -k 10 900 python3 -u bench.py --shape c5 $x --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 2 --warmup 1 --detail gpurun_out/r5f_c5full_${m}_detail.json > gpurun_out/r5f_c5full_${m}.json 2> gpurun_out/r5f_c5full_${m}.log; rc=$?
  tail -2 gpurun_out/r5f_c5full_${m}.log; head -c 1200 gpurun_out/r5f_c5full_${m}.json; echo
  case $rc in 0) ;; *) exit $rc;; esac
done
