# Full GPU suite + smoke + default bench line.
set -o pipefail
tag=${1:-full}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
tail -3 gpurun_out/${tag}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -2 gpurun_out/${tag}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -5 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read())
print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['pipeline'], d['cpu_baseline']['value'], d['timings_s'], d['frame_sha256'][:16])" gpurun_out/${tag}_bench.json
timeout -k 10 300 python bench.py --no-cpu-baseline --multi library --gpus 1 > gpurun_out/${tag}_lib1.json 2> gpurun_out/${tag}_lib1.err || { tail -5 gpurun_out/${tag}_lib1.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read())
print('lib1', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['multi_gpu'], d['frame_sha256'][:16])" gpurun_out/${tag}_lib1.json
