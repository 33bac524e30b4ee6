#!/bin/bash
# Round 3: the default bench line (C2: e2e leg, CPU baseline, in-run PMC traffic) + rocprofv3
# kernel stats of the same workload, then C3 / C4 / C5 with kernel stats.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3/final
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
timeout -k 10 500 python -u bench.py > gpurun_out/r3/final/bench.json 2> gpurun_out/r3/final/bench.err || { echo "bench failed"; tail -20 gpurun_out/r3/final/bench.err; exit 1; }
cat gpurun_out/r3/final/bench.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3/final/prof" -o run --output-format csv -- \
   python -u "$R/bench.py" --no-cpu-baseline --no-traffic --no-e2e --steps 10 --warmup 2 > "$R/gpurun_out/r3/final/bench_prof.json" 2> "$R/gpurun_out/r3/final/bench_prof.err") || { echo "prof failed"; exit 1; }
for c in c3 c4 c5; do
  CFG=$c OUTDIR=r3/final/$c bash tools/gpu_ab.sh - || exit 1
done
OUTDIR=r3/final/pmc_c2 bash tools/gpu_abpmc.sh - > gpurun_out/r3/final/pmc_c2.txt 2>&1 || { echo "pmc failed"; tail gpurun_out/r3/final/pmc_c2.txt; exit 1; }
cat gpurun_out/r3/final/pmc_c2.txt
