#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc run per counter group), kernel-trace/stats only.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out/${OUT:-pmc}"; mkdir -p "$O"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
ARGS="--no-cpu-baseline --no-traffic --steps 2 --warmup 0 --n-res ${NRES:-1000000} ${EXTRA}"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --stats -d "$O" -o pass$i --output-format csv -- \
      python -u "$R/bench.py" $ARGS > "$O/pass$i.json" 2> "$O/pass$i.err" || { echo "pass $i failed"; exit 1; }
done
cd "$R"
for f in $(find "$O" -name "*counter_collection.csv"); do echo "== $f"; python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float)  # (kernel, dispatch, counter) -> value summed over dimensions
for r in rows:
    k = r.get("Kernel_Name", "")
    if k.startswith(("kv_", "kvj_")) and "kv_expand_rows" not in k:
        agg[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
per = collections.defaultdict(list)
for (k, d, c), v in agg.items():
    per[(k, c)].append(v)
tot = collections.defaultdict(float)
for (k, c), v in sorted(per.items()):
    m = sum(v) / len(v)
    tot[c] += m
    print(f"{k} {c}: dispatches={len(v)} mean={m:.6g}")
for c, v in sorted(tot.items()):
    print(f"PER-STEP (sum of kernel means) {c}: {v:.6g}")
PY
done
