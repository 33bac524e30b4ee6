#!/bin/bash
# Round 3 final: GPU tests + smoke, then the default bench line, rocprofv3 kernel stats,
# C3 / C4 / C5 and the C2 PMC counters (kernels from the in-tree code-object cache).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
bash tools/gpu_r3t.sh || exit 1
bash tools/gpu_r3b2.sh || exit 1
