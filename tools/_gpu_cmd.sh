cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 python3 -u tools/step_ab.py --key 8 --values 0 1 --rounds 3 > gpurun_out/r02q_ab_sv.log 2>&1 && \
timeout -k 10 300 python3 -u tools/step_ab.py --key 8 --values 0 1 --rounds 3 --k 50 --agents-per-axis 2 > gpurun_out/r02q_ab_sv_share.log 2>&1
