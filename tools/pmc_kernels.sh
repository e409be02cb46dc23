cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rm -rf gpurun_out/pmck_f gpurun_out/pmck_w && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmck_f -o f -- python3 tools/bench_kernels.py > gpurun_out/pmck_f.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmck_w -o w -- python3 tools/bench_kernels.py > gpurun_out/pmck_w.log 2>&1 && \
python3 tools/pmc_summary.py gpurun_out/pmck_f gpurun_out/pmck_w "k_combine<2, float, 8, 2, 1>" sum_f32_k8_nt 33554432 301989888 gpurun_out/pmc_c3.json && \
python3 tools/pmc_summary.py gpurun_out/pmck_f gpurun_out/pmck_w "k_combine<5, unsigned long, 8, 1, 1>" band_u64_k4_nt 268435456 1342177280 gpurun_out/pmc_c4.json && \
python3 tools/pmc_summary.py gpurun_out/pmck_f gpurun_out/pmck_w "k_combine<11, mvx::pfi, 8, 1, 1>" maxloc_float_int_k8_nt 67108864 603979776 gpurun_out/pmc_c5.json
