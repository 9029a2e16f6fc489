cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && \
timeout -k 10 400 python3 -u bench.py > gpurun_out/r02m_bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02m -o run -- python3 bench.py --cpu-baseline 0 > gpurun_out/r02m_ktrace_bench.log 2>&1 && \
python3 tools/rocpd_stats.py gpurun_out/prof_r02m --timed-steps 20 > gpurun_out/r02m_cg_timed_kernel_stats.csv 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02m_share -o run -- python3 bench.py --k 50 --agents-per-axis 2 --cpu-baseline 0 > gpurun_out/r02m_ktrace_share.log 2>&1 && \
python3 tools/rocpd_stats.py gpurun_out/prof_r02m_share --timed-steps 20 > gpurun_out/r02m_share_timed_kernel_stats.csv 2>&1 && \
timeout -k 10 700 python3 tools/pmc_step.py run gpurun_out/pmc_r02m > gpurun_out/r02m_pmc_run.log 2>&1 && \
python3 tools/pmc_step.py summarize gpurun_out/pmc_r02m > gpurun_out/r02m_pmc_traffic.json 2> gpurun_out/r02m_pmc_sum.err && \
find gpurun_out/prof_r02m gpurun_out/prof_r02m_share gpurun_out/pmc_r02m -name '*.db' -delete
