set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "philox or stat or kat or fast" > gpurun_out/gputest_px.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest_px.log; [ $rc = 0 ] || exit 1
bash scripts/ab.sh nr-ray-tracer_amd/ab/base/libnrt.so nr-ray-tracer_amd/nrt/libnrt.so 3 --steps 10 --warmup 2 || exit 1
bash scripts/ab.sh nr-ray-tracer_amd/ab/base/libnrt.so nr-ray-tracer_amd/nrt/libnrt.so 2 --scene scenes/utah-teapot-scene.json --steps 3 --warmup 1 || exit 1
bash scripts/ab.sh nr-ray-tracer_amd/ab/base/libnrt.so nr-ray-tracer_amd/nrt/libnrt.so 2 --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64 --steps 3 --warmup 1 || exit 1
