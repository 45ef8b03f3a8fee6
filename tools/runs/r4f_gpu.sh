# C5 schedule evidence on the one GPU: the C5 shard (1.25M users) on one rank at 2 epoch-chunks
# (625k users per chunk, C5's 16 chunks over 10M users), and the same shard as C5@8 over 8 gloo
# ranks at 2 chunks (the committed rehearsal line profiles/r4_gloo8_c5.json)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
B="python -u bench.py --shape c5 --users 1250000 --steps 1 --warmup 0 --rmse-epochs 20 --no-cpu-baseline --no-svdpp --no-predict"
timeout -k 10 400 $B --chunks 2 > gpurun_out/r4f_c5shard_c2.json 2> gpurun_out/r4f_c5shard_c2.log || exit $?
grep '^{' gpurun_out/r4f_c5shard_c2.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('shard 1 rank c2', r['rmse'])"
timeout -k 10 500 $B --gpus 8 --backend gloo --chunks 2 > gpurun_out/r4_gloo8_c5.json 2> gpurun_out/r4_gloo8_c5.log || exit $?
grep '^{' gpurun_out/r4_gloo8_c5.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); ph=r['roofline']['phases_gpu_ms']; print('c5@8 c2', r['rmse'], ph.get('allreduce_ms_per_chunk'), ph.get('allreduce_bytes_per_chunk'))"
