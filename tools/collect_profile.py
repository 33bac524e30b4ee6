#!/usr/bin/env python3
"""Copy one GPU round's measurements from gpurun_out/ into profiles/<name>/ and derive
per-pass HBM traffic from the PMC passes (MI355X_MICROARCH.md HBM section: FETCH_SIZE
and WRITE_SIZE are KB; on gfx950 FETCH_SIZE counts half the bytes of 16 B/lane
coalesced reads, so it is doubled; WRITE_SIZE is exact for such stores).

    python tools/collect_profile.py r01_v4
"""
import csv
import collections
import json
import os
import shutil
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_pass(csv_path, counter):
    """Sum over the validate kernels of one pass of their mean per-dispatch counter value."""
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(csv_path)):
        k = r.get("Kernel_Name", "")
        # the pass's kernels; the record-compaction kernels (kv::kv_rec_*) run once per fetch,
        # outside the timed passes (the e2e leg of the same command)
        if r["Counter_Name"] == counter and k.startswith(("kv_", "kvj_", "kv::")) and "kv_rec_" not in k \
                and "kv_expand_rows" not in k:
            agg[(k, r["Dispatch_Id"])] += float(r["Counter_Value"])
    per_k = collections.defaultdict(list)
    for (k, _), v in agg.items():
        per_k[k].append(v)
    return sum(sum(v) / len(v) for v in per_k.values())


def main():
    name = sys.argv[1]
    src = os.path.join(R, "gpurun_out")
    dst = os.path.join(R, "profiles", name)
    os.makedirs(dst, exist_ok=True)
    copies = {"bench_full.json": "bench.json", "bench_prof.json": "bench_under_rocprof.json",
              "gpu_tests.log": "gpu_tests.log", "smoke.log": "smoke.log", "pmc.txt": "pmc.txt",
              "prof/run_kernel_stats.csv": "kernel_stats.csv"}
    for s, d in copies.items():
        if os.path.exists(os.path.join(src, s)):
            shutil.copy(os.path.join(src, s), os.path.join(dst, d))
    pmc = os.path.join(src, "pmc")
    fetch = write = None
    for i in range(1, 5):
        f = os.path.join(pmc, f"pass{i}_counter_collection.csv")
        if not os.path.exists(f):
            continue
        shutil.copy(f, os.path.join(dst, f"pass{i}_counter_collection.csv"))
        heads = {r["Counter_Name"] for r in csv.DictReader(open(f))}
        if "FETCH_SIZE" in heads:
            fetch = per_pass(f, "FETCH_SIZE")
        if "WRITE_SIZE" in heads:
            write = per_pass(f, "WRITE_SIZE")
    bench = json.loads(open(os.path.join(dst, "bench.json")).read().strip().splitlines()[-1])
    run_id = name
    try:  # the gpurun call that produced these files: its verdict file's time
        import datetime

        t = os.path.getmtime(os.path.join(src, ".last_call.json"))
        run_id = f"{name} @ {datetime.datetime.utcfromtimestamp(t).strftime('%Y-%m-%dT%H:%M:%SZ')}"
    except OSError:
        pass
    if fetch is not None and write is not None:
        traffic = 2 * fetch * 1024 + write * 1024
        out = {"workload": bench["config"]["workload"], "resources_per_gpu": bench["config"]["resources_per_gpu"],
               "rules": bench["config"]["rules"], "output": bench["config"]["output"],
               "engine": bench["config"]["engine"],
               "fetch_size_kb": fetch, "write_size_kb": write, "bytes_per_pass": traffic,
               "algorithmic_bytes_per_pass": bench["roofline"]["bytes_per_launch"],
               "source": f"profiles/{name}/pass*_counter_collection.csv (2 x FETCH_SIZE + WRITE_SIZE, KB->B)",
               "run_id": run_id}
        json.dump(out, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
