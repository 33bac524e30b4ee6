set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r1/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r1/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r1/gpu_tests.log
timeout -k 10 500 python -u bench.py > gpurun_out/r1/bench.json 2> gpurun_out/r1/bench.err || { echo "bench failed"; tail -20 gpurun_out/r1/bench.err; exit 1; }
cat gpurun_out/r1/bench.json
