#!/bin/bash
# Read-request size classes of a bench config's kernels (rocprofv3 --pmc, one pass of four TCC
# counters): bytes = 128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B against FETCH_SIZE.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; A=gpurun_out/${OUT:-rdreq}; mkdir -p $A
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
(cd /tmp && timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum \
   --kernel-trace --stats -d "$R/$A/rq" -o rq --output-format csv -- \
   python -u "$R/bench.py" --config ${CFG:-c2} --steps 2 --warmup 0 --no-cpu-baseline --no-e2e --no-traffic \
   > "$R/$A/rq.json" 2> "$R/$A/rq.err") || { echo "rdreq pass failed"; tail -5 $A/rq.err; exit 1; }
python - $A <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/rq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if k.startswith(("kvj_", "kv_", "kv::")):
            agg[(k[:28], r["Counter_Name"])] += float(r["Counter_Value"]); n[(k[:28], r["Counter_Name"])].add(r["Dispatch_Id"])
ks = sorted(set(k for k, _ in agg))
for k in ks:
    g = lambda c: agg.get((k, c), 0.0) / max(1, len(n.get((k, c), {0})))
    b = 128 * g("TCC_EA0_RDREQ_128B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + 32 * g("TCC_EA0_RDREQ_32B_sum")
    tot = g("TCC_EA0_RDREQ_sum"); cls = g("TCC_EA0_RDREQ_128B_sum") + g("TCC_EA0_RDREQ_64B_sum") + g("TCC_EA0_RDREQ_32B_sum")
    print(f"  {k:28s} read {b / 1e9:7.3f} GB/dispatch  req {tot:.4g} (classes {cls:.4g}: 128B {g('TCC_EA0_RDREQ_128B_sum'):.3g} 64B {g('TCC_EA0_RDREQ_64B_sum'):.3g} 32B {g('TCC_EA0_RDREQ_32B_sum'):.3g})")
PY
