set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r02n_gpu.log 2>&1; echo "gpu rc=$?"; tail -12 gpurun_out/r02n_gpu.log
