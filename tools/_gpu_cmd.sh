cd $GRAFT_REPO_ROOT && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02o_gputest.log 2>&1 && \
timeout -k 10 300 python3 -u tools/step_ab.py --key 5 --values 0 1 --rounds 2 > gpurun_out/r02o_ab.log 2>&1 && \
timeout -k 10 300 python3 -u tools/step_ab.py --key 5 --values 0 1 --rounds 2 --k 50 --agents-per-axis 2 > gpurun_out/r02o_ab_share.log 2>&1
