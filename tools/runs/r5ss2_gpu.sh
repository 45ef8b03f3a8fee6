#!/bin/bash
# round 5: the split step's side-stream policy (engine.SIDE_STREAM_POLICY) -- 10 engines per
# policy in a fresh process each (tools/probes/headline_bimodal.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -f gpurun_out/r5ss2_side.jsonl
for pol in pool cached cached-high high; do
  timeout -k 10 240 python -u tools/probes/headline_bimodal.py gpurun_out/r5ss2_side.jsonl $pol > gpurun_out/r5ss2_$pol.log 2>&1; rc=$?
  echo "$pol rc $rc"; [ $rc -eq 0 ] || exit $rc
done
python - <<'PY'
import json
for l in open("gpurun_out/r5ss2_side.jsonl"):
    r = json.loads(l); print(r["policy"], r["n"], r["dtype"], r["ms_per_step"], round(r["replay_ms"], 4))
PY
