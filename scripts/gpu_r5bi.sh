# Two groups per queue atomic for the KF_FLAT kernels (current) vs the last commit; parity first.
set -o pipefail
L=nr-ray-tracer_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_stat_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bi_pytest.log 2>&1 || { tail -30 gpurun_out/r5bi_pytest.log; exit 1; }
tail -1 gpurun_out/r5bi_pytest.log
timeout -k 10 1000 python scripts/ab_configs.py --reps 3 --steps 20 --timeout 200 --out gpurun_out/r5bi_ab.jsonl \
  --arm cur=$L/nrt/libnrt.so --arm prev=$L/ab/prev/libnrt.so \
  --cfg c5="" --cfg c4="--scene scenes/utah-teapot-scene.json" --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128"
