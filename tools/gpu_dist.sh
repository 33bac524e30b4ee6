#!/bin/bash
# GPU tests + C5 scopes bench + a 2-rank rehearsal of the multi-GPU bench path (gloo, both ranks on one GPU).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/dist
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 2 > gpurun_out/dist/c5_scopes.json 2> gpurun_out/dist/c5_scopes.err || { echo "c5 failed"; tail gpurun_out/dist/c5_scopes.err; exit 1; }
cat gpurun_out/dist/c5_scopes.json
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --n-res 200000 --config c5 --backend gloo > gpurun_out/dist/rehearsal.json 2> gpurun_out/dist/rehearsal.err || { echo "rehearsal failed"; tail -20 gpurun_out/dist/rehearsal.err; exit 1; }
cat gpurun_out/dist/rehearsal.json
