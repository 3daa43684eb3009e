# Default bench (3 frames in flight) + multi-GPU tests + the headline profile of the default command.
set -o pipefail
tag=${1:-r5o}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_multigpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -5 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read())
print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['pipeline']['frames_in_flight'], d['cpu_baseline']['value'], d['frame_sha256'][:16])" gpurun_out/${tag}_bench.json
rm -rf gpurun_out/prof_r05_c5_f32_philox
bash scripts/profile.sh r05_c5_f32_philox --steps 20 --warmup 5 || exit 1
python3 scripts/trace_period.py gpurun_out/prof_r05_c5_f32_philox/trace --json gpurun_out/prof_r05_c5_f32_philox/trace_period.json
