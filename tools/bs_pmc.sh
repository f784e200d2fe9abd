# bitsliced ctr pass: kernel trace + SQ counters (one pass each), gcm_bs=${MODE-1}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="python3 $R/bench.py --steps 10 --warmup 5 --no-cpu --no-e2e --no-inplace-leg --no-encrypt-leg --tuning gcm_bs=${MODE-1}"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bsp_trace -o run --output-format csv -- $B > $R/gpurun_out/bsp_trace.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU -d $R/gpurun_out/bsp_sq -o run --output-format csv -- $B > $R/gpurun_out/bsp_sq.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d $R/gpurun_out/bsp_sq2 -o run --output-format csv -- $B > $R/gpurun_out/bsp_sq2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/bsp_fetch -o run --output-format csv -- $B > $R/gpurun_out/bsp_fetch.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/bsp_write -o run --output-format csv -- $B > $R/gpurun_out/bsp_write.log 2>&1
