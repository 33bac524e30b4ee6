#!/bin/bash
# Round 3: host ingest phases on the GPU box (pinned store allocation included)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_VERBOSE=1
timeout -k 10 300 python -u tools/ingest_phases.py 1000000 > gpurun_out/r3/ingest_phases.log 2>&1
grep -E "ingest|Pods" gpurun_out/r3/ingest_phases.log
