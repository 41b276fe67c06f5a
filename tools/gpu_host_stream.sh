set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload rebuild_stream_8p2 --steps 5 --warmup 1 > gpurun_out/host1.log 2>&1 || exit $?
tail -1 gpurun_out/host1.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --workload rebuild_stream_8p2 --gpus 2 --steps 5 --warmup 1 > gpurun_out/host2.log 2>&1 || exit $?
grep '^{' gpurun_out/host2.log
timeout -k 10 300 python bench.py --workload dec_8p2 --steps 10 --warmup 2 --no-cpu > gpurun_out/dec8p2.log 2>&1 || exit $?
grep '^{' gpurun_out/dec8p2.log | cut -c1-600
