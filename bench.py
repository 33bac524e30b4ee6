#!/usr/bin/env python3
"""Benchmark: resource x rule validate.pattern evaluations per second (BASELINE.json).

One step = one pass of the hot path over one batch: every (resource, rule) pair
of the config evaluated on the GPU (match/exclude prefilter + pattern VM +
verdict output), inputs resident in HBM. Default workload = config C2
(1M synthetic Pods x 100 pattern rules per GPU). Multi-GPU: one process per
GPU, each evaluates its own shard of resources (weak scaling, no data-path
collective); per-rule pass/fail/... counts are all-reduced over RCCL once after
the timed region (PolicyReport summary), outside the timing.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n-res R] [--mode full|counts|scopes] [--config c2|c3|c4|c5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# code objects of the configs' specialized kernels, compiled ahead of time (tools/jit_warm.sh)
os.environ.setdefault("KVGPU_JIT_CACHE", os.path.join(ROOT, "kyverno_amd", "jitcache"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
KV_LANES_CHUNK = 65536  # smallest e2e_stream chunk


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu() -> dict:
    """Host core count (all cores, and those this process may run on) and the CPU model (lscpu)."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    quota = None
    try:  # cgroup v2 CPU quota ("max" = none)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    usable = min(avail, quota) if quota else avail
    return {"nproc": os.cpu_count() or 1, "affinity": avail, "cgroup_quota_cores": quota, "available": usable,
            "model": model}


def cpu_baseline(policies, pairs: float, threads: int, kind_mix: int = 0, label: str = "C2") -> dict:
    """Oracle (CPU restatement of the reference engine) on a bounded sample of the same workload:
    the first resources of the benchmark's synthetic stream, about `pairs` resource x rule pairs."""
    import oracle
    from kyverno_amd import batch, workloads

    orc = oracle.get()
    n_rules = sum(len(p["spec"]["rules"]) for p in policies)
    n_sample = max(1000, int(pairs // max(1, n_rules)))
    data = batch.synth(workloads.SEED, n_sample, kind_mix).strip()
    st, secs = orc.validate_ndjson(json.dumps(policies), data, nthreads=threads, preparse=True)
    n_rules = st.shape[0]
    return {"value": n_sample * n_rules / secs, "unit": "resource×rule evals/s", "cores": threads,
            "host": host_cpu(), "kind": "port",
            "sample": f"first {n_sample} resources of the benchmark stream x {n_rules} rules ({label} rule set), "
                      f"evaluation only (inputs pre-parsed), oracle/ C++ restatement on {threads} host threads, "
                      f"{secs:.2f} s"}


def pmc_traffic(args) -> dict | None:
    """HBM bytes per pass of this workload from rocprofv3 PMC counters, measured by this command:
    two child runs of this script, one counter group each (kernel-trace/stats only): the L2's
    memory-side read requests by size class (TCC_EA0_RDREQ_128B / _64B / _32B: bytes = 128 / 64 / 32
    per request; FETCH_SIZE tallies a 128-byte request at 64 B, MI355X_MICROARCH.md HBM section) and
    WRITE_SIZE. Per kernel the counters are averaged over its dispatches (every kernel of a pass runs
    once per pass), then summed over the pass's kernels (not the record compaction of a fetch,
    kv_rec_*, nor the row expansion and path-column build that run once per batch)."""
    import csv
    import collections
    import glob
    import shutil
    import signal
    import subprocess
    import tempfile

    rp = shutil.which("rocprofv3")
    if not rp:
        return None
    # not when this process already runs under a profiler (its preloaded library has initialised
    # the GPU here; a nested rocprofv3 would exec from a GPU-initialised process)
    if "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ):
        log("pmc: running under a profiler, in-run traffic skipped")
        return None
    out = tempfile.mkdtemp(prefix="kvpmc.", dir=os.environ.get("TMPDIR", "/tmp"))
    child = [sys.executable, "-u", os.path.abspath(__file__), "--config", args.config, "--n-res", str(args.n_res),
             "--mode", args.mode, "--engine", args.engine, "--steps", "2", "--warmup", "0", "--no-cpu-baseline",
             "--no-e2e", "--no-traffic"]
    groups = {"read": {"TCC_EA0_RDREQ_128B_sum": 128, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_32B_sum": 32},
              "write": {"WRITE_SIZE": 1024}}
    vals = {}
    for name, ctrs in groups.items():
        launcher = [sys.executable, rp] if open(rp, "rb").read(2) == b"#!" else [rp]
        cmd = launcher + ["--pmc", *ctrs, "--kernel-trace", "--stats", "-d", out, "-o", name, "--output-format", "csv",
                          "--"] + child
        p = subprocess.Popen(cmd, cwd=out, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, start_new_session=True)
        try:
            _, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            log(f"pmc {name}: timed out")
            return None
        if p.returncode != 0:
            log(f"pmc {name}: rocprofv3 exit {p.returncode}: {err.decode(errors='replace')[-400:]}")
            return None
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for f in sorted(set(glob.glob(os.path.join(out, "**", f"{name}*counter_collection.csv"), recursive=True))):
            for r in csv.DictReader(open(f)):
                k = r.get("Kernel_Name", "")
                if r["Counter_Name"] in ctrs and k.startswith(("kv_", "kvj_", "kv::")) and "kv_rec_" not in k \
                        and "kv_expand_rows" not in k and "kv_pcol_" not in k:
                    agg[k] += float(r["Counter_Value"]) * ctrs[r["Counter_Name"]]
                    disp[k].add(r.get("Dispatch_Id", ""))
        if not agg:
            return None
        vals[name] = {k: v / max(1, len(disp[k])) for k, v in agg.items()}
    shutil.rmtree(out, ignore_errors=True)
    fetch = sum(vals["read"].values())
    write = sum(vals["write"].values())
    return {"bytes_per_pass": fetch + write, "read_bytes": fetch, "write_bytes": write,
            "per_kernel_read": dict(sorted(vals["read"].items())),
            "run_id": f"in-run PMC, pid {os.getpid()}, {time.strftime('%Y-%m-%dT%H:%M:%SZ', time.gmtime())}"}


def ingest_parts(ps, args, kind_mix: int, mode: int):
    """Parts session of --gpus N in one process: shard k (resources [k*N, (k+1)*N) of the stream)
    synthesized and ingested by a worker thread (ctypes calls release the GIL; at most
    KVGPU_BENCH_INFLIGHT shards in flight, default 2), attached to device k (device 0 for
    --parts-per-gpu rehearsals) and dropped. Returns (session, per-shard info, t_start, t_end)."""
    import concurrent.futures as cf

    from kyverno_amd import batch, workloads

    G = args.gpus
    inflight = max(1, int(os.environ.get("KVGPU_BENCH_INFLIGHT", "2")))
    sess = batch.Session.parts(ps, G, mode=mode)

    def make(k):
        data = batch.synth(workloads.SEED, args.n_res, kind_mix, first=k * args.n_res)
        nb = len(data)
        t = time.time()
        b = batch.Batch(ps, data)
        return k, b, nb, time.time() - t

    info = [None] * G
    t1 = time.time()
    with cf.ThreadPoolExecutor(max_workers=inflight) as ex:
        pending = set()
        nxt = 0
        while nxt < G or pending:
            while nxt < G and len(pending) < inflight:
                pending.add(ex.submit(make, nxt))
                nxt += 1
            done, pending = cf.wait(pending, return_when=cf.FIRST_COMPLETED)
            for f in done:
                k, b, nb, secs = f.result()
                dev = 0 if args.parts_per_gpu > 1 else k
                sess.attach_part(k, b, dev)
                info[k] = {"n_res": b.n_res, "store_bytes": b.store_bytes, "ndjson_bytes": nb, "ingest_s": secs,
                           "device": dev}
                b.close()  # the session holds the device copy
    t2 = time.time()
    return sess, info, t1, t2


def check_rccl(ranks: int, devices) -> None:
    """The in-process parts session must reduce its counts over one RCCL rank per distinct device
    (kv_session_rccl_ranks = ncclCommCount); parts that all share one device sum on the host
    (0 ranks). Anything else means the multi-device path is not the one being measured."""
    distinct = len(set(devices))
    want = distinct if distinct > 1 else 0
    if ranks != want:
        raise SystemExit(f"bench: RCCL communicator has {ranks} ranks, expected {want} "
                         f"({distinct} distinct devices among {len(devices)} parts)")


def e2e_stream(ps, n_res: int, kind_mix: int, device: int, seed: int, chunk: int, ingesters: int = 4) -> dict:
    """Ingest-inclusive rate of a caller streaming NDJSON through the C ABI: the batch is cut into
    chunks; four host workers ingest chunks side by side (kv_ingest, a quarter of the host
    threads each: one's serial phases overlap the others' parallel ones) while the chunks already ingested are
    uploaded, evaluated and fetched (kv_validate: H2D of the page-locked store, one pass, D2H of
    statuses and compacted records, the dense status matrix built on the host) on two more
    threads (ctypes calls release the GIL). Timed from the first NDJSON byte to the last chunk's
    results on the host."""
    import concurrent.futures as cf

    from kyverno_amd import batch

    chunks = [batch.synth(seed, min(chunk, n_res - k), kind_mix, first=k) for k in range(0, n_res, chunk)]
    mode = batch.MODE_STATUS | batch.MODE_ERRORS
    t_ing, t_val = [0.0], [0.0]
    inflight = 2  # chunks being uploaded / evaluated / fetched (and `ingesters` chunks being ingested)
    threads = int(os.environ.get("KVGPU_INGEST_THREADS", min(16, os.cpu_count() or 1)))
    per = max(1, threads // ingesters)

    def ingest(data):
        t = time.perf_counter()
        b = batch.Batch(ps, data)
        t_ing[0] += time.perf_counter() - t
        return b

    def evaluate(b):
        t = time.perf_counter()
        r = batch.validate(ps, b, device=device, mode=mode, copy=False)
        _ = r.status  # the dense status matrix on the host (materialised from the transfer form)
        t_val[0] += time.perf_counter() - t
        return r

    saved = os.environ.get("KVGPU_INGEST_THREADS")
    os.environ["KVGPU_INGEST_THREADS"] = str(per)  # (read by each kv_ingest call)
    try:
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(max_workers=ingesters) as ix, cf.ThreadPoolExecutor(max_workers=inflight) as vx:
            ing = [ix.submit(ingest, d) for d in chunks[:ingesters]]
            nxt, val, done = ingesters, [], 0
            while ing:
                b = ing.pop(0).result()
                if nxt < len(chunks):
                    ing.append(ix.submit(ingest, chunks[nxt]))
                    nxt += 1
                while len(val) >= inflight:
                    val.pop(0).result()
                    done += 1
                val.append(vx.submit(evaluate, b))
                del b
            for f in val:
                f.result()
                done += 1
        secs = time.perf_counter() - t0
    finally:
        if saved is None:
            os.environ.pop("KVGPU_INGEST_THREADS", None)
        else:
            os.environ["KVGPU_INGEST_THREADS"] = saved
    n_rules = ps.n_rules
    return {"seconds": secs, "evals_per_s": n_res * n_rules / secs, "resources_per_s": n_res / secs,
            "chunks": len(chunks), "chunk_resources": chunk, "in_flight": inflight, "ingesters": ingesters,
            "ingest_threads_each": per, "ingest_seconds": t_ing[0], "validate_seconds": t_val[0],
            "includes": "NDJSON -> kv_ingest (four chunks at a time, a quarter of the host threads each) overlapped with "
                        "kv_validate of the chunks ingested before (H2D + pass + D2H of statuses and records + "
                        "the dense status matrix, two in flight)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-res", type=int, default=None,
                    help="resources per GPU (default: the config's per-GPU share at 8 GPUs: C2/C4 1M, "
                         "C3 10M/8, C5 50M/8)")
    ap.add_argument("--mode", choices=["full", "counts", "scopes"], default=None,
                    help="full: status + failing-path records per pair; counts: per-rule histogram only; "
                         "scopes: per-namespace PolicyReport counts (status kept on device). "
                         "Default: full, scopes for c5")
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2: Pods x 100 pattern rules; c3: mixed kinds x 1000 policies with match/exclude; "
                         "c4: anchor-heavy chart + test/policy/validate + status forms (142 rules) x Pods; "
                         "c5: background scan, chart after autogen (105 rules) x mixed kinds, counts")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive kv_validate timing")
    ap.add_argument("--stream-ingesters", type=int, default=4,
                    help="e2e_stream: chunks ingested side by side (the host threads split among them)")
    ap.add_argument("--cpu-pairs", type=float, default=6e7,
                    help="resource x rule pairs of the CPU baseline sample (~10 s on 16 EPYC cores at C2)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default=None,
                    help="torch.distributed backend for N>1 (default: nccl = RCCL when GPUs are visible); "
                         "gloo lets several ranks share one GPU for a rehearsal")
    ap.add_argument("--rule-filter", default="", help="diagnostics: regex over C2 rule names")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the PMC traffic measurement (two rocprofv3 --pmc child runs of this workload)")
    ap.add_argument("--engine", choices=["vm", "specialized"], default="specialized",
                    help="bytecode interpreter kernel, or per-policy-set specialized kernels (hiprtc)")
    ap.add_argument("--parts-per-gpu", type=int, default=1,
                    help="in-process multi-device path only: run each device's share as this many logical "
                         "parts on device 0 (KVGPU_SHARDS_PER_DEVICE; rehearses --gpus N on one GPU)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    # --gpus N without a launcher (no WORLD_SIZE): one process drives the N devices through the
    # library's own multi-device session (kv_session_create_devices: one host thread + stream per
    # device, per-rule counts all-reduced over RCCL inside libkvgpu). Under torch.distributed.run
    # (WORLD_SIZE set) every rank is one process on one GPU and evaluates its own shard.
    inproc = "WORLD_SIZE" not in os.environ and args.gpus > 1
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist  # noqa: F811

        backend = args.backend or ("nccl" if torch.cuda.device_count() > 0 else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
        local = local % max(1, torch.cuda.device_count())

    from kyverno_amd import batch, report, workloads

    if args.config == "c2":
        pols = workloads.c2_policies()
        if args.rule_filter:  # diagnostics only: evaluate a subset of the C2 rules
            import re

            rx = re.compile(args.rule_filter)
            for p in pols:
                p["spec"]["rules"] = [r for r in p["spec"]["rules"] if rx.search(r["name"])]
        kind_mix = 0
        workload = "C2: synthetic Pods x 100 validate.pattern rules (image globs, ?*, quantities, |-lists)"
    elif args.config == "c3":
        pols = workloads.c3_policies(1000)
        kind_mix = workloads.C3_KIND_MIX  # 1 000 namespaces
        workload = "C3: Pods/Deployments/Services 60/25/15 over 1000 namespaces x 1000 policies with match/exclude"
    elif args.config == "c4":
        pols = workloads.c4_policies()
        kind_mix = 0
        workload = "C4: anchor-heavy kyverno-policies chart (restricted) + test/policy/validate, autogen, x Pods"
    else:
        pols = workloads.c5_policies()
        kind_mix = 1
        workload = "C5: background scan, kyverno-policies chart (restricted) after autogen x Pods/Deployments/Services"
    if args.mode is None:
        args.mode = "scopes" if args.config == "c5" else "full"
    if args.n_res is None:
        args.n_res = {"c2": 1_000_000, "c3": 10_000_000 // 8, "c4": 1_000_000, "c5": 50_000_000 // 8}[args.config]
    t0 = time.time()
    os.environ.setdefault("KVGPU_PROGRESS", "1")  # hiprtc progress lines on stderr during long compiles
    ps = batch.PolicySet(pols, specialize=args.engine == "specialized")
    jit = ps.jit_info
    if jit["kernels"]:
        log(f"[rank {rank}] specialized kernels: {jit['kernels']} ({jit['code_bytes'] / 1e3:.0f} KB code), "
            f"hiprtc {jit['compile_ms'] / 1e3:.1f}s")
    mode = {"full": batch.MODE_STATUS | batch.MODE_ERRORS, "counts": batch.MODE_COUNTS,
            "scopes": batch.MODE_COUNTS | batch.MODE_SCOPES}[args.mode]
    # rank r evaluates the contiguous shard [r * N, (r + 1) * N) of one synthetic stream
    n_devs = args.gpus if inproc else 1
    if inproc:
        # one process drives the N devices (kv_session_create_parts): device k's shard
        # [k * N, (k + 1) * N) is synthesized and ingested on its own (a few shards in flight),
        # uploaded to its device and dropped, so the host never holds the node's whole batch
        if args.parts_per_gpu > 1 and args.parts_per_gpu != args.gpus:
            raise SystemExit("--parts-per-gpu must equal --gpus (all parts on device 0)")
        sess, shard_info, t1, t2 = ingest_parts(ps, args, kind_mix, mode)
        n_res_total = sum(x["n_res"] for x in shard_info)
        store_bytes = sum(x["store_bytes"] for x in shard_info)
        ndjson_bytes = sum(x["ndjson_bytes"] for x in shard_info)
        namespaces = sess.scope_names() if args.mode == "scopes" else []
        b = None
        log(f"in-process multi-device session: {sess.n_parts} parts, RCCL ranks {sess.rccl_ranks()}")
        check_rccl(sess.rccl_ranks(), [x["device"] for x in shard_info])
    else:
        data = batch.synth(workloads.SEED, args.n_res, kind_mix, first=rank * args.n_res)
        ndjson_bytes = len(data)
        # a long-running caller page-locks its store / result arena once at startup (kv_host_reserve),
        # not inside the first batch's ingest: about 2.5x the NDJSON for the store, plus the status
        # matrix and records of a FULL fetch
        reserve = int(2.5 * ndjson_bytes) + (10 * ps.n_rules * args.n_res if args.mode == "full" else 0)
        batch.host_reserve(min(reserve, 96 << 30))
        t1 = time.time()
        b = batch.Batch(ps, data)
        t2 = time.time()
        del data  # (the caller's input buffer; its release is not ingest work)
        n_res_total, store_bytes, namespaces = b.n_res, b.store_bytes, b.namespaces
        # device-resident session: inputs uploaded and output buffers allocated once (untimed)
        sess = batch.Session(ps, b, device=local, mode=mode)
    log(f"[rank {rank}] compile+synth {t1 - t0:.2f}s ingest {t2 - t1:.2f}s store {store_bytes / 1e6:.1f} MB "
        f"({store_bytes / n_res_total:.0f} B/resource), rules {ps.n_rules}")
    sess.run(1)
    counts = sess.counts()
    n_fail = int(counts[:, 1].sum() + counts[:, 3].sum() + counts[:, 4].sum())
    if args.warmup > 0:
        sess.run(args.warmup)
    if dist is not None:
        dist.barrier()
    ts = time.perf_counter()
    event_ms = sess.run(args.steps)  # K passes on the session stream, waited for (device sync)
    te = time.perf_counter()
    if dist is not None:
        dist.barrier()
    wall = te - ts
    kernel_ms = event_ms / args.steps
    # The K timed passes re-validate the resident batch: pass i + 1's per-pass tables are built on a
    # low-priority stream beside pass i's rule kernels (DESIGN.md §4 Streams). A caller validating
    # each batch once runs one pass with its tables in order: single_pass_ms (median of 5, untimed
    # for `value`).
    single = sorted(sess.run(1) for _ in range(5))
    single_ms = single[len(single) // 2]
    status_written = sess.status_bytes() if args.mode == "full" else 0
    t_max = wall
    if dist is not None:
        import torch

        t = torch.tensor([wall], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_max = float(t.item())
    # PolicyReport summaries (outside the timed region): per-rule counts, and in scopes mode the
    # per-namespace counts, summed over the ranks with one all-reduce each (RCCL / gloo)
    counts = report.allreduce_counts(counts, dist)
    scopes = None
    if args.mode == "scopes":
        names, sc = report.allreduce_scope_counts(namespaces, sess.scope_counts(len(namespaces)), dist)
        summ = report.scope_summaries(ps.rules, pols, names, sc)
        scopes = {"reports": len(summ), "fail": sum(v["fail"] for v in summ.values()),
                  "pass": sum(v["pass"] for v in summ.values())}

    n_gpus = n_devs * world
    rehearsal = inproc and args.parts_per_gpu > 1  # G logical parts on one physical device
    n_pairs_rank = n_res_total * ps.n_rules // n_devs  # per GPU
    value = n_gpus * n_pairs_rank * args.steps / t_max
    # algorithmic bytes per launch: projected store read once + program tables + outputs
    prog_bytes = 0  # program/predicate tables are KB-scale (<0.01%)
    # full: 1 B status + 8 B compact error record per FAIL/ERROR/SKIP pair (kvdevtypes.h ErrRec8;
    # the rare records that do not fit also write 32 B, not counted); scopes: the 4 B scope index of
    # every resource (the rule kernels count per scope inside the pass; the per-scope counts
    # themselves are KB-scale)
    # (full: the status bytes the pass wrote — a 256-resource segment of a rule whose statuses are all
    # NOMATCH is not written but flagged, and filled at fetch; kv_session_status_bytes)
    out_bytes = {"full": status_written // n_devs + 8 * n_fail // n_devs, "counts": 0,
                 "scopes": 4 * n_res_total // n_devs}[args.mode]
    b_alg = store_bytes // n_devs + prog_bytes + out_bytes  # per GPU (the slowest part's event time below)
    achieved = b_alg / (kernel_ms / 1e3) / 1e9
    traffic, traffic_src = None, None  # filled below by the in-run PMC measurement (rank 0, N=1)
    out = {
        "metric": "resource×rule validate evals/sec (node)",
        "value": value,
        "unit": "evals/s",
        "n_gpus": 1 if rehearsal else n_gpus,
        "parts": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic (kv_synth_range, seed 0x6B79766E, rank shard [r*N, (r+1)*N), N={args.n_res})",
        "config": {"workload": workload, "resources_per_gpu": n_res_total // n_devs, "rules": ps.n_rules,
                   "pairs_per_gpu": n_pairs_rank, "output": args.mode,
                   "parallelism": (f"resource-shard x{n_gpus} (one process, kv_session_create_parts: per-device "
                                   f"ingest, RCCL count all-reduce in libkvgpu"
                                   + (f", {args.parts_per_gpu} logical parts on device 0)" if args.parts_per_gpu > 1
                                      else ")")) if inproc else f"resource-shard x{world}",
                   "engine": args.engine},
        "kernel_ms_per_step": kernel_ms,
        "pipelined": True,
        "single_pass_ms": single_ms,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "bytes_per_launch": b_alg, "bytes_per_eval": b_alg / n_pairs_rank,
                     "output_bytes": out_bytes, "status_bytes_written": status_written // n_devs,
                     "single_pass_frac": b_alg / (single_ms / 1e3) / 1e9 / HBM_PEAK_GBS},
        "status_counts": {n: int(counts[:, i].sum()) for i, n in enumerate(batch.STATUS_NAMES)},
    }
    if scopes is not None:
        out["policy_reports"] = scopes
    # which RCCL reduces the PolicyReport counts: the communicator inside libkvgpu (in-process
    # parts on distinct devices; 0 ranks = host sum of logical parts), or torch.distributed
    if inproc:
        out["rccl"] = {"ranks": sess.rccl_ranks(), "where": "libkvgpu ncclCommInitAll",
                       "devices": sorted(set(x["device"] for x in shard_info)),
                       "part_ms": [m / args.steps for m in sess.part_ms()],
                       "part_ingest_s": [x["ingest_s"] for x in shard_info]}
    elif dist is not None:
        out["rccl"] = {"ranks": world if dist.get_backend() == "nccl" else 0,
                       "where": f"torch.distributed ({dist.get_backend()})"}
    # host ingest (NDJSON -> projected columnar store, kv_ingest; multi-threaded), outside `value`
    out["ingest"] = {"seconds": t2 - t1, "resources_per_s": n_res_total / (t2 - t1),
                     "MB_per_s": ndjson_bytes / (t2 - t1) / 1e6,
                     "threads": int(os.environ.get("KVGPU_INGEST_THREADS", min(16, os.cpu_count() or 1)))}
    if rank == 0 and n_gpus == 1 and args.mode == "full" and not args.no_e2e:
        # PCIe-inclusive rate of the host boundary: kv_validate on a freshly ingested
        # batch = H2D upload of the projected store + one pass + D2H of statuses and error records
        sess = None
        # steady state of a host that validates batch after batch: one untimed kv_validate on another
        # batch first (the library keeps its pinned staging / result buffers), then the timed one on a
        # freshly ingested batch
        bw = batch.Batch(ps, batch.synth(workloads.SEED + 7, args.n_res, kind_mix))
        rw = batch.validate(ps, bw, device=local, copy=False)
        del rw, bw
        b2 = batch.Batch(ps, batch.synth(workloads.SEED, args.n_res, kind_mix, first=rank * args.n_res))
        xfer = b2.transfer_bytes
        te0 = time.perf_counter()
        r2 = batch.validate(ps, b2, device=local, copy=False)  # statuses stay in the result's pinned buffer
        te1 = time.perf_counter()
        _ = r2.status  # the dense caller-order matrix, materialised on the host from the transfer form
        te2 = time.perf_counter()
        out["e2e_kv_validate"] = {"seconds": te1 - te0, "evals_per_s": n_pairs_rank / (te1 - te0),
                                  "kernel_ms": r2.kernel_ms,
                                  "phases_ms": {k: round(v, 3) for k, v in r2.phases.items()},
                                  "status_matrix_ms": round(1e3 * (te2 - te1), 3),
                                  "upload_bytes": xfer, "upload_bytes_per_resource": round(xfer / args.n_res, 1),
                                  "includes": "H2D store upload + 1 pass + D2H statuses (transfer form: the "
                                              "segments the pass wrote, 4 bits a status) and error records "
                                              "(1-byte codes into per-rule tables); status_matrix_ms: the "
                                              "dense [rule][res] matrix built from it on first read (steady "
                                              "state: after one untimed kv_validate of another batch)"}
        del r2, b2
        # the same stream as a caller would push it: ingest overlapped with upload + pass + fetch
        out["e2e_stream"] = e2e_stream(ps, args.n_res, kind_mix, local, workloads.SEED + 13,
                                       max(KV_LANES_CHUNK, args.n_res // 16), args.stream_ingesters)
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline:
        # every core this process may run on (the GPU box grants a share of the machine's cores;
        # nproc and the CPU model are recorded beside it)
        threads = host_cpu()["available"]
        out["cpu_baseline"] = cpu_baseline(pols, args.cpu_pairs, threads, kind_mix, args.config.upper())
    if rank == 0 and n_gpus == 1 and not args.no_traffic:
        # measured HBM bytes of the same workload (child rocprofv3 --pmc runs), after this
        # process's device buffers are freed
        sess = None
        import gc

        gc.collect()
        t = pmc_traffic(args)
        if t is not None:
            out["roofline"]["traffic"] = t["bytes_per_pass"]
            out["roofline"]["traffic_source"] = t["run_id"] + (" (TCC_EA0_RDREQ 128B/64B/32B x size + WRITE_SIZE, "
                                                               "rocprofv3 --pmc, per dispatch)")
            out["roofline"]["traffic_over_alg"] = t["bytes_per_pass"] / b_alg
            out["roofline"]["traffic_detail"] = {"read": t["read_bytes"], "write": t["write_bytes"],
                                                 "per_kernel_read": t["per_kernel_read"]}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
