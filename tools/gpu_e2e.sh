#!/bin/bash
# e2e (PCIe-inclusive kv_validate) phases of configs $CFGS under env variants (args: "K=V,K2=V2" or "-"),
# then (TRACE=1) one rocprofv3 kernel + memory-copy + HIP API trace of the first config. Output under gpurun_out/$OUT.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/${OUT:-e2e}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
for c in ${CFGS:-c2}; do
  for spec in "$@"; do
    envs=""; [ "$spec" != "-" ] && envs=$(echo "$spec" | tr ',' ' ')
    tag=$(echo "$c.$spec" | tr -c 'A-Za-z0-9.\n' '_')
    env $envs timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-traffic $BENCH_ARGS \
      > $O/$tag.json 2> $O/$tag.err || { echo "bench $c $spec failed"; tail -5 $O/$tag.err; exit 1; }
    python - "$O/$tag.json" "$c $spec" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
e = d.get("e2e_kv_validate", {}); s = d.get("e2e_stream", {})
print(sys.argv[2], "pass %.4f ms" % d["kernel_ms_per_step"], "e2e %.1f ms" % (1e3 * e.get("seconds", 0)),
      "stream %.3g evals/s" % s.get("evals_per_s", 0), "ingest %.3g res/s" % d["ingest"]["resources_per_s"])
print("   ", e.get("phases_ms"))
PY
  done
done
if [ -n "$TRACE" ]; then
  c=$(echo ${CFGS:-c2} | cut -d' ' -f1)
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --stats -d "$R/$O/trace" \
     -o run --output-format csv -- python -u "$R/bench.py" --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-traffic \
     > "$R/$O/trace.json" 2> "$R/$O/trace.err") || { echo "trace failed"; tail -5 $O/trace.err; exit 1; }
  echo trace ok
fi
