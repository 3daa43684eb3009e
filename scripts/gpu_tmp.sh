set -o pipefail
bash scripts/ab.sh nr-ray-tracer_amd/ab/base/libnrt.so nr-ray-tracer_amd/nrt/libnrt.so 3 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_stat_parity.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r02l_stat.log 2>&1; echo "stat rc=$?"; grep -E "chi2|FAIL|Error" gpurun_out/r02l_stat.log | tail -20
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r02l_gpu.log 2>&1; echo "gpu rc=$?"; tail -5 gpurun_out/r02l_gpu.log
