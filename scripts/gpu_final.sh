# Final check of a round's library: GPU suite, smoke, full-frame JIT/generic comparison, default bench line.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
tag=${1:-final}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -5 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 200 python scripts/jit_compare.py > gpurun_out/${tag}_jit_compare.log 2>&1; rc=$?; tail -3 gpurun_out/${tag}_jit_compare.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench_default.json 2> gpurun_out/${tag}_bench_default.err || exit 1
tail -c 400 gpurun_out/${tag}_bench_default.json
