#!/bin/bash
# Round 3: GPU test suite + smoke, then the kind-first rule order A/B on C3 / C5.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
bash tools/gpu_r3t.sh || exit 1
bash tools/gpu_r3i.sh || exit 1
