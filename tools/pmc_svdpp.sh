# usage (on the GPU box): bash tools/pmc_svdpp.sh TAG [extra bench args, e.g. --shape c5 --users
# 1250000] -- counter passes over the SVD++ C3 bench step
# (mf_svdpp_hx_kernel + the y fold): the q-row atomics at the L2 (TCC) and at the memory side (EA),
# the EA atomic latency accumulator, and where the waves' cycles go (SQ).  One --pmc pass per
# counter group; a pass that is killed or faults ends the script, an unknown counter only its pass.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pp}
shift
B="bench.py --no-cpu-baseline --no-rmse --algo svdpp --mode atomic --steps 5 --warmup 1 $*"
i=0
for pass in "TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum" "TCC_EA0_ATOMIC_LEVEL_sum TCC_EA0_ATOMIC_sum" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $pass -T --output-format csv -d gpurun_out/pmc_${TAG}_$i -o run -- python3 $B > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i ($pass): exit $rc"
  case $rc in 0|1|2) ;; *) exit $rc ;; esac
done
