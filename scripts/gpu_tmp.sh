bash scripts/profile.sh r1list --steps 1 --warmup 1 --precision f32 --rng philox && python3 scripts/pmc_summary.py gpurun_out/prof_r1list > gpurun_out/prof_r1list/summary.json
