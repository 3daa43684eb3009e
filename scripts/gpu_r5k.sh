set -o pipefail
tag=${1:-r5k}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_multigpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest.log
for r in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --multi library --gpus 1 > gpurun_out/${tag}_lib1.json 2> gpurun_out/${tag}_lib1.err || { tail -5 gpurun_out/${tag}_lib1.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read())
print('lib1', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['multi_gpu']['frame_ms_gpu0'], d['frame_sha256'][:16])" gpurun_out/${tag}_lib1.json
done
