#!/bin/bash
# PMC A/B of kernel variants: for each argument (env list "K=V,K2=V2", "-" for none) one
# rocprofv3 --pmc pass per counter group of a short bench ($CFG, default c2): FETCH_SIZE, WRITE_SIZE,
# L2 hits / misses, and the SQ wave / instruction / wait counters; prints per-kernel means per dispatch.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; A=gpurun_out/${OUTDIR:-abpmc}; mkdir -p $A
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=""; [ "$spec" != "-" ] && envs=$(echo "$spec" | tr ',' ' ')
  j=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"; do
    j=$((j+1))
    (cd /tmp && env $envs timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace --stats -d "$R/$A/v$i" -o pass$j --output-format csv -- \
       python -u "$R/bench.py" --config ${CFG:-c2} --steps 2 --warmup 0 --no-cpu-baseline --no-e2e --no-traffic ${BENCH_ARGS} \
       > "$R/$A/v$i.pass$j.json" 2> "$R/$A/v$i.pass$j.err") || { echo "pmc $spec pass $j failed"; tail -5 $A/v$i.pass$j.err; exit 1; }
  done
  echo "== $spec"
  python - $A/v$i <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if k.startswith(("kvj_", "kv_")) and "kv_expand_rows" not in k and "kv_rec_" not in k:
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for (k, c), v in sorted(agg.items()):
    m = v / len(n[(k, c)])
    if c == "FETCH_SIZE": m = 2 * m * 1024  # KB, gfx950 half-counted (MI355X_MICROARCH.md)
    if c == "WRITE_SIZE": m = m * 1024
    print(f"  {k[:22]:22s} {c:18s} {m:.4g}")
PY
done
