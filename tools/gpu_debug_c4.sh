set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/debug_c4.py 3000 || exit 1
KVGPU_JIT_WAVES=0 timeout -k 10 120 python tools/debug_c4.py 3000 || exit 1
KVGPU_JIT_GROUP=1 timeout -k 10 120 python tools/debug_c4.py 3000 || exit 1
