cd $GRAFT_REPO_ROOT && \
timeout -k 10 400 python3 -u bench.py > gpurun_out/r02s_bench.log 2>&1
