bash scripts/profile.sh r1v2 --steps 1 --warmup 1 --precision f32 --rng chacha8
