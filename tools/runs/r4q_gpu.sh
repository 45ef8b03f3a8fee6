# experiment: the lookahead body's bank of rows (MF_LA_BANK, one lane group: fp32 K <= 127 and the
# C4 layout) at 8 (product), 16 and 4 -- C4 (SVD K=128 fp32) and ML-1M fp32
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
C4="python3 -u bench.py --shape c4 --steps 5 --warmup 2 --no-rmse --no-cpu-baseline --no-chain-probe"
ML="python3 -u bench.py --dtype f32 --steps 50 --warmup 5 --no-rmse --no-cpu-baseline --no-chain-probe --no-svdpp --no-predict --no-c4"
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; print('$1', round(r['ms_per_step'],4), {k: round(v,3) for k, v in ph.items() if k.endswith('_ms')})"; }
for v in prod bank16 bank4; do
  if [ $v = prod ]; then L=""; else L="SURPRISE_AMD_LIB=$GRAFT_REPO_ROOT/surprise_amd/variants/libsurprise_amd_$v.so"; fi
  env $L timeout -k 10 300 $C4 > gpurun_out/r4q_c4_$v.json 2> gpurun_out/r4q_c4_$v.log || exit $?; show r4q_c4_$v
  env $L timeout -k 10 120 $ML > gpurun_out/r4q_ml_$v.json 2> gpurun_out/r4q_ml_$v.log || exit $?; show r4q_ml_$v
done
