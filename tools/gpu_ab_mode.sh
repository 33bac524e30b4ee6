set -o pipefail
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_fuzz_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/fuzz.log 2>&1 || { tail -30 gpurun_out/ab/fuzz.log; exit 1; }
tail -2 gpurun_out/ab/fuzz.log
for m in full counts; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 --mode $m > gpurun_out/ab/b_$m.json 2> gpurun_out/ab/b_$m.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab/b_$m.json'));print('$m', d['value'], d['kernel_ms_per_step'])"
done
