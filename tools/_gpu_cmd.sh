cd $GRAFT_REPO_ROOT && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02p_gputest.log 2>&1 && \
timeout -k 10 300 python3 -u tools/step_ab.py --key 7 --values 1 0 --rounds 3 > gpurun_out/r02p_ab_lookahead.log 2>&1 && \
timeout -k 10 300 python3 -u tools/step_ab.py --key 7 --values 1 0 --rounds 3 --k 50 --agents-per-axis 2 > gpurun_out/r02p_ab_lookahead_share.log 2>&1
