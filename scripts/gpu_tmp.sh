set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_multigpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02m_mgpu.log 2>&1; echo "mgpu rc=$?"; tail -15 gpurun_out/r02m_mgpu.log
