cd $GRAFT_REPO_ROOT && \
DPGO_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --k 48 --burnin 20 --cpu-baseline 0 > gpurun_out/r02n_bench_2rank_rehearsal.log 2>&1
