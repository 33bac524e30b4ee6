#!/bin/bash
# Kernel trace + stats of a short bench run (config $CFG, output gpurun_out/$OUT): per-kernel times, grid, registers, LDS.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out/${OUT:-prof}"; mkdir -p "$O"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O" -o run --output-format csv -- python -u "$R/bench.py" --config ${CFG:-c2} --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$O/bench.json" 2> "$O/bench.err" || exit 1
f=$(find "$O" -name "*kernel_stats.csv" | head -1); cat "$f" | cut -d, -f1-8 | head -20
f=$(find "$O" -name "*kernel_trace.csv" | head -1); python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
seen = {}
for r in rows:
    k = r["Kernel_Name"]
    if k not in seen:
        seen[k] = r
for k, r in seen.items():
    print(k, "grid", r.get("Grid_Size_X", r.get("Grid_Size")), r.get("Grid_Size_Y", ""), "wg", r.get("Workgroup_Size_X", ""), "vgpr", r.get("Arch_VGPR_Count", r.get("VGPR_Count", "")), "sgpr", r.get("SGPR_Count", ""), "lds", r.get("LDS_Block_Size", r.get("Lds_Size", "")), "scratch", r.get("Scratch_Size", r.get("Private_Segment_Size", "")))
PY
