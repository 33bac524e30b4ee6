#!/bin/bash
# SQ issue / wait breakdown of the rule kernels (one rocprofv3 --pmc pass per counter group, short
# bench of $CFG): prints per-kernel means per dispatch. Output under gpurun_out/$OUT.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; A=gpurun_out/${OUT:-sqpmc}; mkdir -p $A
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
j=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS" $EXTRA; do
  j=$((j+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --stats -d "$R/$A/g$j" -o pass --output-format csv -- \
     python -u "$R/bench.py" --config ${CFG:-c2} --steps 2 --warmup 0 --no-cpu-baseline --no-e2e --no-traffic $BENCH_ARGS \
     > "$R/$A/g$j.json" 2> "$R/$A/g$j.err") || { echo "pmc group $j failed"; tail -5 $A/g$j.err; exit 1; }
done
python - $A <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if k.startswith("kvj_r"):
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for (k, c), v in sorted(agg.items()):
    print(f"  {k[:22]:22s} {c:22s} {v / len(n[(k, c)]):.4g}")
PY
