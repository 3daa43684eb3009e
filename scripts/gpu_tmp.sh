# scratch GPU script (varies per experiment): GPU tests, then the round profile + default bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pytest.log 2>&1 || { tail -30 gpurun_out/t_pytest.log; exit 1; }
tail -2 gpurun_out/t_pytest.log
bash scripts/round_profile.sh ${1:-r01e}
