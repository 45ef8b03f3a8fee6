# rocprofv3 kernel trace + stats of the default bench command itself (the driver's line)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r4t_default -o run -- python3 -u bench.py > gpurun_out/r4t_default_bench.json 2> gpurun_out/r4t_default_bench.log || exit $?
head -12 gpurun_out/prof_r4t_default/run_kernel_stats.csv | cut -c1-160
