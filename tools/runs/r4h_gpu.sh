# Why does the full C5 (10M users) cost 2.4x more per rating than the C5 shard (1.25M users)?
# Epoch time against the user count and the chunking, and a kernel trace of the full workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python -u bench.py --shape c5 --no-rmse --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 2 --warmup 1"
show() { grep '^{' gpurun_out/$1.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; ek=ph['epoch_kernel']; print('$1', r['config']['workload'][-60:], round(r['ms_per_step'],2), 'epoch', round(ph['epoch_kernel_ms'],2), 'launches', ek['launches']['all']['per_step'], round(ek['launches']['all']['avg_us'],1), 'yfold', round(ph['replay_ms'],2))"; }
timeout -k 10 300 $B --users 1250000 > gpurun_out/r4h_u1250k.json 2> gpurun_out/r4h_u1250k.log || exit $?; show r4h_u1250k
timeout -k 10 300 $B --users 1250000 --chunks 13 > gpurun_out/r4h_u1250k_c13.json 2> gpurun_out/r4h_u1250k_c13.log || exit $?; show r4h_u1250k_c13
timeout -k 10 400 $B --users 5000000 > gpurun_out/r4h_u5m.json 2> gpurun_out/r4h_u5m.log || exit $?; show r4h_u5m
timeout -k 10 500 $B --chunks 16 > gpurun_out/r4h_full_c16.json 2> gpurun_out/r4h_full_c16.log || exit $?; show r4h_full_c16
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r4h_full -o run -- python3 -u bench.py --shape c5 --no-rmse --no-cpu-baseline --no-svdpp --no-predict --no-c4 --no-chain-probe --steps 2 --warmup 1 > gpurun_out/r4h_full.json 2> gpurun_out/r4h_full.log || exit $?; show r4h_full
