# bitsliced ctr pass knob breakdown (knobs library; results broken on purpose)
ESPGPU_LIB=$PWD/f-stack_amd/libespgpu_knobs.so timeout -k 10 200 python tools/gcm_timing.py --tuning gcm_bs=1 --opts 0 128 256 512 384 896 > gpurun_out/bs_knobs.jsonl 2>&1
timeout -k 10 100 python tools/gcm_timing.py --opts 0 > gpurun_out/bs_knobs_fused.jsonl 2>&1
