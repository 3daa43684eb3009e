rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
bash scripts/profile.sh r1base --steps 1 --warmup 1 --precision f32 --rng chacha8
