#!/usr/bin/env python3
"""Benchmark: sealed-segment DataExpr evaluation on MI355X (BASELINE.json metric, config C2).

One step = one evaluation of the query over every HBM-resident segment of this GPU's shard (scan kernel +
finalize/compaction + result copy back to the host), i.e. one `lk_eval_pushdown` / `lk_eval_pushdown_dist`
call.  Weak scaling: every GPU holds `--segments` segments of `--rows` rows (C2: 64 x 2^24); at N > 1 the
request names all N x 64 segments, each rank scans its shard and the partial tables meet on rank 0 over RCCL.

    python bench.py                      # N=1, C2
    python bench.py --gpus 8             # N=8: this process starts the 8 rank processes itself (one per GPU)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port P bench.py --gpus 8
    python bench.py --gpus 2 --comm host # rehearsal: 2 ranks on one GPU over the host transport

At N > 1 every rank times the CPU restatement on its own shard and sends its partial cells to rank 0, which folds
them with query-api semantics and checks the merged GPU rows against them (`validated`); `cpu_baseline` is the
whole workload's rows over the slowest rank's shard time.
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "rows/sec scanned + datapoints/sec emitted, 1B-row sealed DataExpr eval"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)

QUERIES = {
    # C2 (BASELINE.json configs[1]): single :eq tag + :sum at 1m step
    "c2": dict(filter={"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq", "extracted": False,
                       "computed": False, "dataType": "string"}, agg="sum", group_bys=[],
               desc=":eq _cardinalhq.name=metric_07 :sum, step 1m"),
    # C2 at the step query-api picks for windows <= 65 min (QueryApi.scala:297-300): 10 s buckets, so nearly every
    # 64K-row tile straddles bucket boundaries and the zone maps cannot spare the timestamp column
    "c2s10": dict(filter={"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq", "extracted": False,
                          "computed": False, "dataType": "string"}, agg="sum", group_bys=[], step=10000,
                  desc=":eq _cardinalhq.name=metric_07 :sum, step 10s"),
    # C2 over real values (SURVEY §8(d) "real" mode, lognormal(0, 2)): no load-time "integral" summary applies, so every
    # SUM add takes the compensated double-double path (the <= 1 ulp bar of north_star)
    "c2real": dict(filter={"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq", "extracted": False,
                           "computed": False, "dataType": "string"}, agg="sum", group_bys=[], value_mode=1,
                   desc=":eq _cardinalhq.name=metric_07 :sum, step 1m, lognormal(0,2) values (compensated sums)"),
    # C2 with the timestamps permuted within each 1M-row row group: no tile is sorted (no split tile) and no tile is
    # pinned to one bucket by its zone map, so every passing row gathers its timestamp (the sortedness-free C2)
    "c2shuf": dict(filter={"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq", "extracted": False,
                           "computed": False, "dataType": "string"}, agg="sum", group_bys=[], ts_shuffle=1,
                   desc=":eq _cardinalhq.name=metric_07 :sum, step 1m, timestamps shuffled within each row group"),
    # C3 (configs[2]): :and/:re multi-tag predicate + :by 2-key group-by :max
    "c3": dict(filter={"op": "and",
                       "q1": {"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq"},
                       "q2": {"k": "resource.service.name", "v": ["^svc-0[0-4]"], "op": "regex"}},
               agg="max", group_bys=["resource.service.name", "resource.k8s.namespace.name"],
               desc=":and(:eq name, :re service ^svc-0[0-4]) :by service,namespace :max, step 1m"),
    # C4 (configs[3], per GPU): :eq name :sum :by service (an unrestricted group dim: at N > 1 the ranks agree on
    # the sorted union of their dictionaries before the scan)
    "c4": dict(filter={"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq", "extracted": False,
                       "computed": False, "dataType": "string"}, agg="sum", group_bys=["resource.service.name"],
               desc=":eq _cardinalhq.name=metric_07 :sum :by resource.service.name, step 1m"),
    # C4 over real values (compensated sums into 24,000 cells)
    "c4real": dict(filter={"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq", "extracted": False,
                           "computed": False, "dataType": "string"}, agg="sum", group_bys=["resource.service.name"],
                   value_mode=1,
                   desc=":eq _cardinalhq.name=metric_07 :sum :by resource.service.name, step 1m, lognormal(0,2) values"),
    # C5 (configs[4]): 10M-value group key, all segments in hour 0, one 1h bucket (<= 10M datapoints); 8 segments
    # per GPU (64 over the node)
    "c5": dict(filter={"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq", "extracted": False,
                       "computed": False, "dataType": "string"}, agg="sum", group_bys=["resource.container.id"],
               step=3600000, hour=0, highcard_n=10_000_000, segments=8,
               desc=":eq _cardinalhq.name=metric_07 :sum :by resource.container.id (10M-value dictionary), step 1h"),
    # tag query (§8(f) f4) on C2 data: values of resource.service.name among metric_07's rows, with COUNT(*)
    # (query-api's `IS NOT NULL` on the tag included); reads the name + service columns only
    "tag": dict(filter={"op": "and", "q1": {"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq"},
                        "q2": {"k": "resource.service.name", "v": [], "op": "exists"}},
                agg="count", group_bys=[], tag="resource.service.name",
                desc="tag query resource.service.name where :eq _cardinalhq.name=metric_07, COUNT(*)"),
    # exemplar raw scan (§8(f) f4) on C2 data: per glob the newest 1000 rows of metric_07 (ORDER BY ts DESC LIMIT 1000)
    "exemplar": dict(filter={"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq", "extracted": False,
                             "computed": False, "dataType": "string"}, agg=None, group_bys=[], exemplar=1000,
                     desc="exemplar :eq _cardinalhq.name=metric_07, ORDER BY ts DESC LIMIT 1000 per glob"),
    # numeric comparison leaf on the value column: scan_lean filters on the name and tests the
    # value of every passing row (BaseExpr.scala:488-498)
    "gt": dict(filter={"op": "and", "q1": {"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq"},
                       "q2": {"k": "_cardinalhq.value", "v": ["1.5"], "op": "gt", "dataType": "number"}},
               agg="sum", group_bys=[], desc=":and(:eq _cardinalhq.name=metric_07, :gt _cardinalhq.value 1.5) :sum, step 1m"),
    # C2's filter with COUNT: name codes only (no value column read for a NULL-free value column; zone-map buckets),
    # the single-column scan_lean's filter + accumulate cost on its own (beside the tag query's one late column)
    "count": dict(filter={"k": "_cardinalhq.name", "v": ["metric_07"], "op": "eq", "extracted": False,
                          "computed": False, "dataType": "string"}, agg="count", group_bys=[],
                  desc=":eq _cardinalhq.name=metric_07 :count, step 1m"),
    # every row passes: reads every timestamp/value (calibrates the PMC byte counters against a known count)
    "dense": dict(filter={"k": "_cardinalhq.name", "v": [f"metric_{i:02d}" for i in range(16)], "op": "in",
                          "extracted": False, "computed": False, "dataType": "string"}, agg="sum", group_bys=[],
                  desc=":in _cardinalhq.name=<all 16> :sum, step 1m"),
}


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _visible_gpus():
    """GPUs this job can see, counted in a child process so that this launcher never initialises the GPU itself (it
    starts the rank processes afterwards)."""
    import subprocess
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        log(f"could not count GPUs: {r.stderr.strip()[-500:]}")
        return 0


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): start N rank processes of this script, one per
    GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them), before any GPU call here, and
    exit with the worst rank status.  Fewer visible GPUs than N is an error with RCCL (one rank per device); the
    host transport (--comm host) puts every rank on GPU 0 (a rehearsal of the N-rank protocol on one GPU)."""
    import signal
    import subprocess
    n = args.gpus
    ndev = _visible_gpus()
    if args.comm == "rccl" and ndev < n:
        log(f"error: --gpus {n} needs {n} visible GPUs (one rank per GPU over RCCL), {ndev} visible; "
            f"use --comm host to rehearse {n} ranks on one GPU")
        return 2
    if ndev < 1:
        log("error: no GPU visible")
        return 2
    if args.comm == "host" and n > 16:
        log("error: at most 16 ranks may share one GPU")
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LK_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    log(f"launched {n} rank processes (pids {[p.pid for p in procs]}, comm {args.comm}, {ndev} GPUs visible)")
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0:
                    rc = rc or c
                    log(f"rank process {p.pid} exited with {c}: stopping the others")
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:   # our own children only, by pid
            if p.poll() is None:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
    return 1 if rc and rc < 0 else rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--segments", type=int, default=None, help="segments per GPU (default: the query's config)")
    ap.add_argument("--rows", type=int, default=1 << 24, help="rows per segment")
    ap.add_argument("--query", default=None, choices=sorted(QUERIES),
                    help="default: c2 (BASELINE configs[1]) at N=1, c4 (configs[3]: :sum :by service, 64 segments "
                         "per GPU) at N > 1")
    ap.add_argument("--cpu-sample", type=int, default=-1,
                    help="segments per rank timed on the CPU restatement (-1: all = full-size validation; 0: skip)")
    ap.add_argument("--gen-workers", type=int, default=4)
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                    help="N > 1 exchange: RCCL over xGMI (default), or the host transport over gloo (rehearsal of the "
                         "multi-rank path with several ranks on one GPU; RCCL refuses two ranks on one device)")
    ap.add_argument("--dist-loopback", action="store_true",
                    help="N=1 only: evaluate through lk_eval_pushdown_dist on a world-1 RCCL communicator with "
                         "LK_COMM_LOOPBACK=1, so every collective of the N > 1 path (all-gathers, grouped "
                         "ncclSend/ncclRecv of the table reduce or the key-range all-to-all) runs on this GPU")
    args = ap.parse_args()

    if args.query is None:
        args.query = "c4" if args.gpus > 1 else "c2"
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world} (the launcher started a different number of ranks)")
        sys.exit(2)

    import torch
    import torch.distributed as dist
    from lakeside_amd import LK_MERGED, LK_PLAN_BYTES, synth
    from lakeside_amd.evaluator import Engine

    if world > 1:
        dist.init_process_group("gloo")
    loopback = args.dist_loopback and world == 1
    if args.dist_loopback and world > 1:
        log("note: --dist-loopback applies at N=1 only; ignored")
    if loopback:
        os.environ["LK_COMM_LOOPBACK"] = "1"   # read by lk_comm_init
    if args.comm == "rccl" and local_rank >= torch.cuda.device_count():
        log(f"error: rank {rank} (local rank {local_rank}) has no GPU of its own: "
            f"{torch.cuda.device_count()} visible")
        sys.exit(2)
    device = local_rank if args.comm == "rccl" else 0
    torch.cuda.set_device(device)
    eng = Engine(device)
    if world > 1 and args.comm == "host":
        eng.comm_init_host(world, rank)
    elif world > 1:
        obj = [Engine.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        eng.comm_init(obj[0], world, rank)
    elif loopback:
        eng.comm_init(Engine.unique_id(), 1, 0)
    use_dist = world > 1 or loopback
    comm_desc = eng.stats.get("comm") if use_dist else None
    if use_dist:
        log(f"rank {rank}: communicator {comm_desc}")

    # ---- segments of this rank (weak scaling: rank r owns global segments [r*S, (r+1)*S)) ----
    q = QUERIES[args.query]
    S = args.segments or q.get("segments", 64)
    step, hour, highcard = q.get("step", 60000), q.get("hour"), q.get("highcard_n", 0)
    total = S * world
    mine = range(rank * S, (rank + 1) * S)
    keys = [f"seg/{i}" for i in range(total)]
    shard = [i // S for i in range(total)]

    def gen(i):
        return i, synth.make_segment(synth.segment_spec(i, rows=args.rows, threads=4, hour=hour,
                                                        highcard_n=highcard, value_mode=q.get("value_mode", 0),
                                                        ts_shuffle=q.get("ts_shuffle", 0)))

    # The CPU baseline / validator reads the same Parquet bytes: every rank keeps its shard in host memory.
    keep_cpu = args.cpu_sample != 0
    kept = {}
    t0 = time.time()
    bytes_loaded = 0
    load_s = 0.0   # disk->HBM load alone (footer + page walk + run tables + remap + upload), synthesis excluded
    with cf.ThreadPoolExecutor(args.gen_workers) as ex:
        for n, fut in enumerate(cf.as_completed([ex.submit(gen, i) for i in mine])):
            i, seg = fut.result()
            tl = time.perf_counter()
            eng.put_segment_ptr(keys[i], seg.ptr, seg.size)
            load_s += time.perf_counter() - tl
            bytes_loaded += seg.size
            if keep_cpu:
                kept[i] = seg
            else:
                seg.free()
            if n % 8 == 7 or S <= 16:
                log(f"rank {rank}: {n + 1}/{S} segments generated + loaded to HBM ({time.time() - t0:.0f}s)")
    log(f"rank {rank}: {S} segments ({bytes_loaded / 1e9:.1f} GB Parquet) resident, HBM cache "
        f"{eng.segment_bytes / 1e9:.1f} GB; Parquet -> HBM load {load_s:.2f} s ({bytes_loaded / load_s / 1e9:.2f} GB/s, "
        f"{load_s / S * 1e3:.0f} ms/segment; synthesis + load {time.time() - t0:.0f}s)")

    segs = [synth.segment_request(i, step=step, hour=hour) for i in range(total)]

    def request(seg_reqs):
        if q.get("exemplar"):
            return json.dumps({"baseExpr": {"id": "A", "dataset": "logs", "filter": q["filter"],
                                            "limit": q["exemplar"]}, "segmentRequests": seg_reqs})
        return json.dumps(synth.pushdown(q["filter"], seg_reqs, q["agg"], q["group_bys"], tag=q.get("tag")))

    req = request(segs)
    local_req = request([segs[i] for i in mine])   # this rank's shard alone

    def step(extra=0):
        if use_dist:
            return eng.eval_pushdown_dist(req, keys, shard, 10)
        return eng.eval_pushdown(req, keys, 10, LK_MERGED | extra)

    # Plan bytes (the roofline numerator) are a property of the query and the data: counted by the kernel in one
    # untimed call (LK_PLAN_BYTES costs ~5% of scan time), then the timed steps run without the counter.  Per GPU:
    # this rank's shard alone (the same scan work it does inside the distributed call).
    pbytes = float(eng.eval_pushdown(local_req, [keys[i] for i in mine], 10, LK_MERGED | LK_PLAN_BYTES)
                   .stats.get("plan_bytes", 0))
    for _ in range(args.warmup):
        res = step()
    # Cold evaluation: the request as if never seen -- parse, leaf-outcome, value-key-order and group-dim caches
    # dropped (segments stay resident) -- one call, wall time; then one warm call so the timed steps start warm.
    if world > 1:
        dist.barrier()
    eng.drop_caches()
    tc = time.perf_counter()
    cold = step()
    cold_ms = (time.perf_counter() - tc) * 1e3
    cold_total_ms = cold.stats.get("total_ms")
    cold_stages = {k: cold.stats.get(k) for k in ("plan_ms", "dims_ms", "dims_rebuilt", "scan_ms", "device_ms",
                                                   "reduce_ms", "scan_agreed_ms") if k in cold.stats}
    del cold
    res = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    scan_ms, total_ms, plan_ms, device_ms, alg_bytes, out_rows = [], [], [], [], 0, 0
    launch_ms, sync_ms, alloc_ms, copy_ms, dims_ms, reduce_ms, agreed_ms = [], [], [], [], [], [], []
    texts = []   # each step's stats, parsed after the timed region
    t_start = time.perf_counter()
    for _ in range(args.steps):
        res = step()
        texts.append(res.stats_text())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    for st in map(json.loads, texts):
        scan_ms.append(st["scan_ms"])
        total_ms.append(st["total_ms"])
        plan_ms.append(st.get("plan_ms", 0.0))
        device_ms.append(st.get("device_ms", 0.0))
        launch_ms.append(st.get("launch_ms", 0.0))
        sync_ms.append(st.get("sync_ms", 0.0))
        alloc_ms.append(st.get("alloc_ms", 0.0))
        copy_ms.append(st.get("copy_ms", 0.0))
        dims_ms.append(st.get("dims_ms", 0.0))
        reduce_ms.append(st.get("reduce_ms", 0.0))
        agreed_ms.append(st.get("scan_agreed_ms", 0.0))
        alg_bytes = st.get("algorithmic_bytes", 0)
    out_rows = len(res)
    avg = lambda xs: sum(xs) / len(xs)   # noqa: E731
    per_rank = {"rank": rank, "device": device, "segments": S, "scan_kernel_ms": avg(scan_ms),
                "eval_ms": elapsed * 1e3 / args.steps, "dims_ms": avg(dims_ms), "reduce_ms": avg(reduce_ms),
                "scan_agreed_ms": avg(agreed_ms), "plan_bytes": pbytes, "comm": comm_desc}
    ranks_info = [per_rank]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        o = torch.tensor([out_rows], dtype=torch.int64)
        dist.all_reduce(o, op=dist.ReduceOp.MAX)
        out_rows = int(o.item())
        ranks_info = [None] * world
        dist.all_gather_object(ranks_info, per_rank)
    ms_per_step = elapsed * 1e3 / args.steps
    rows_total = total * args.rows
    value = rows_total / (ms_per_step / 1e3)
    scan_avg = avg(scan_ms)
    # Roofline numerator: the bytes the late-materialized plan must read, counted by the scan kernel (streams it
    # decodes in full + distinct 128-B lines of its per-row gathers + tile metadata), per launch.
    achieved = pbytes / (scan_avg / 1e3) / 1e9
    alg_gbs = alg_bytes / (scan_avg / 1e3) / 1e9
    log(f"rank {rank}: scan kernel {scan_avg:.3f} ms avg (min {min(scan_ms):.3f}), eval {ms_per_step:.3f} ms/step, "
        f"plan bytes {pbytes / 1e9:.2f} GB/launch -> {achieved:.0f} GB/s ({achieved / HBM_PEAK_GBS:.3f} of peak); "
        f"SURVEY algorithmic {alg_bytes / 1e9:.2f} GB -> {alg_gbs:.0f} GB/s; {out_rows} output rows; in the call: "
        f"plan {avg(plan_ms):.2f} ms, device {avg(device_ms):.2f} ms, total {avg(total_ms):.2f} ms" +
        (f"; group-dim agreement {avg(dims_ms):.2f} ms, reduce {res.stats.get('reduce')}, "
         f"emit {res.stats.get('emit')}, reduce stage {avg(reduce_ms):.3f} ms, "
         f"collectives {res.stats.get('collectives')}" if use_dist else "") + f"; cold eval {cold_ms:.2f} ms")

    # measured device-to-device copy rate on this GPU (a stream-copy peak beside the spec peak)
    copy_gbs = None
    if rank == 0:
        a = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        b.copy_(a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        copy_gbs = 2 * 10 * a.numel() / (e0.elapsed_time(e1) / 1e3) / 1e9   # read + write bytes
        del a, b

    cpu, validated = None, None
    if keep_cpu:
        cpu, validated = cpu_baseline_and_validate(args, q, local_req, [kept[i] for i in mine], res, world, rank,
                                                   dist if world > 1 else None)
    for sgm in kept.values():
        sgm.free()

    # HBM traffic of the scan kernel(s) per launch: rocprofv3 FETCH_SIZE / WRITE_SIZE passes over this same bench
    # command (scripts/gpu_bench_prof.sh -> scripts/pmc_traffic.py; separate runs, as counters must be collected
    # alone), committed under profiles/ -- read here only when it profiled this query at this size.
    # Accepted only when that summary was taken with this very library build (sha256 of the loaded .so) and counted
    # the same plan bytes: a PMC pass of an older kernel says nothing about this one, so otherwise traffic is null.
    traffic, traffic_src = None, None
    lib_sha = _lib_sha16()
    pmc_file = None
    for rnd in ("r06", "r05", "r04", "r03", "r02"):   # the newest committed PMC summary of this query
        cand = os.path.join(ROOT, "profiles", f"{rnd}_pmc_{args.query}.json")
        if os.path.exists(cand):
            pmc_file = cand
            break
    if pmc_file:
        pmc = json.load(open(pmc_file))
        if (pmc.get("query") == args.query and pmc.get("lib_sha16") == lib_sha
                and pmc.get("plan_bytes_per_launch") == pbytes and world == 1):
            traffic = pmc["hbm_bytes_per_launch"]
            traffic_src = (f"profiles/{os.path.basename(pmc_file)}: rocprofv3 --pmc FETCH_SIZE (x{pmc['fetch_correction']} "
                           f"gfx950 correction, calibrated in profiles/r02_gather_fetchsize.json) + WRITE_SIZE passes "
                           f"over this bench command with this library build (sha256 {lib_sha}); scan kernel "
                           f"{pmc.get('scan_kernel_ms')} ms in that run")
        else:
            traffic_src = (f"null: the newest PMC summary (profiles/{os.path.basename(pmc_file)}) was taken with "
                           f"library {pmc.get('lib_sha16')} / plan bytes {pmc.get('plan_bytes_per_launch')}, this run "
                           f"is library {lib_sha} / plan bytes {pbytes:.0f}")

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "rows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": f"synthetic sealed Parquet (tools/synth.cpp, seed 20240101+i), {S} x {args.rows} rows per GPU",
            "config": {"workload": f"{args.query.upper()}: {total} segments x {args.rows} rows, {q['desc']}",
                       "segments_per_gpu": S, "rows_per_segment": args.rows, "glob_size": 10,
                       "parallelism": f"segment-sharded x{world}" + ((", RCCL table reduce" if args.comm == "rccl" else ", host-transport table reduce (rehearsal: every rank on GPU 0)") if world > 1 else "")},
            "datapoints_per_sec": out_rows / (ms_per_step / 1e3),
            "load": {"what": "Parquet bytes -> HBM segment cache (lk_segment_put: footer, page walk, run tables, "
                             "dictionary remap, upload), synthetic generation excluded; not in value",
                     "segments": S, "parquet_bytes": bytes_loaded, "seconds": load_s,
                     "gbs": bytes_loaded / load_s / 1e9 if load_s else None,
                     "ms_per_segment": load_s / S * 1e3},
            "rows_scanned": rows_total, "output_rows": out_rows,
            "scan_kernel_ms": scan_avg, "eval_ms": ms_per_step,
            "cold_eval_ms": cold_ms,
            "cold_eval": {"what": "first evaluation of the request after lk_engine_drop_caches (parsed request, "
                                  "leaf outcomes, value-key orders, group-dim unions dropped; segments resident); "
                                  "wall time of the call", "ms": cold_ms, "engine_total_ms": cold_total_ms,
                          "stages": cold_stages},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "definition": "achieved = plan bytes per launch (counted by the scan kernel: streams "
                                       "decoded in full + distinct 128-B lines of every per-row gather + tile "
                                       "metadata) / scan-kernel time (HIP events on the call's stream), rank 0's "
                                       "shard at N > 1. `value` "
                                       "counts every row of the workload as scanned, including rows of tiles whose "
                                       "load-time zone map (timestamp min/max per tile) pins them to a single "
                                       "bucket and of split tiles (timestamps never decreasing: the bucket "
                                       "boundary rows are found by searching them, r05): their timestamps are "
                                       "never gathered per row, and value lines with no passing row are skipped, "
                                       "so plan bytes < SURVEY's algorithmic bytes; a plan change that reads fewer "
                                       "bytes lowers `frac` at equal time -- compare `value` and scan time across "
                                       "rounds",
                         "plan_bytes_per_launch": pbytes,
                         "algorithmic_bytes_per_launch": alg_bytes, "algorithmic_gbs": alg_gbs,
                         "frac_algorithmic": alg_gbs / HBM_PEAK_GBS,
                         "frac_algorithmic_note": "SURVEY §8(d)'s algorithmic bytes (every referenced column chunk in "
                                                  "full) / scan-kernel time / 8 TB/s, beside `frac` (plan bytes): above "
                                                  "1 when the plan skips bytes §8(d) counts (zone-mapped / split-tile "
                                                  "timestamps, value lines with no passing row)",
                         "traffic_source": traffic_src,
                         "traffic_gbs": traffic / (scan_avg / 1e3) / 1e9 if traffic else None,
                         "stream_copy_gbs": copy_gbs},
            "validated": validated,
            "lib_sha16": lib_sha,
            "cpu_baseline": cpu,
        }
        if use_dist:   # the distributed call's own stages (rank 0): group-dim agreement, table reduce, row emission
            line["comm_world"] = (comm_desc or {}).get("world")
            line["dist"] = {"dims_ms": avg(dims_ms), "reduce": res.stats.get("reduce"),
                            "emit": res.stats.get("emit"), "comm": args.comm,
                            "communicator": comm_desc,
                            "loopback": loopback,
                            "scan_agreed_ms": avg(agreed_ms),
                            "reduce_ms": avg(reduce_ms),
                            "collectives_per_query": res.stats.get("collectives"),
                            "allgathers": res.stats.get("allgathers"), "allgather_bytes": res.stats.get("allgather_bytes"),
                            "p2p_groups": res.stats.get("p2p_groups"), "p2p_bytes": res.stats.get("p2p_bytes"),
                            "ranks": ranks_info}
            if loopback:
                line["config"]["parallelism"] = ("segment-sharded x1 through lk_eval_pushdown_dist on a world-1 RCCL "
                                                 "communicator in loopback (every collective of the N>1 path runs)")
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


def _lib_sha16():
    """First 16 hex digits of the sha256 of the evaluator library this process loaded."""
    import hashlib
    from lakeside_amd import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:16]


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_and_validate(args, q, local_req, segs, gpu_res, world=1, rank=0, dist=None):
    """The CPU restatement (oracle/cpu: C++17 + OpenMP over the same in-memory Parquet bytes, the job's CPU share)
    timed on this rank's shard, and the GPU's merged rows checked against it.  A reported baseline, not the target
    (the reference's JVM + DuckDB cannot run here).

    N > 1: every rank evaluates its own shard (concurrently over RCCL -- one rank per GPU, each with its own CPU share
    -- or one rank after another when the ranks share one GPU's CPU share, --comm host) and sends its per-glob partial
    cells to rank 0, which folds them with query-api semantics (TimeGroupedSketchAggregator.scala:74-92: add, min, max
    per (timestamp, tags)) and compares the result with the distributed call's merged rows.  Columnar throughout
    (oracle.cpu.evaluate_cell_table / merge_cell_table, tests.parity.result_columns), so millions of rows (C5) check
    in seconds."""
    from oracle import cpu as lkcpu
    from oracle import dataexpr as dx
    from tests.parity import result_columns
    # The job's CPU share: the affinity mask, capped by OMP_NUM_THREADS where the pool sets it (the GPU box allots
    # 16 host cores per GPU and sets OMP_NUM_THREADS=16; os.cpu_count() there is the whole host).
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(affinity, int(omp)) if omp else affinity
    n = len(segs) if args.cpu_sample < 0 else min(len(segs), args.cpu_sample)
    blobs = [(s.ptr, s.size) for s in segs[:n]]
    body = json.loads(local_req)
    body["segmentRequests"] = body["segmentRequests"][:n]
    pr = dx.parse_pushdown(json.dumps(body))
    agg = q["agg"]
    tag = q.get("tag")
    concurrent = world == 1 or args.comm == "rccl"

    exemplar = q.get("exemplar")

    def evaluate(timing=None):   # tag queries: {tag text -> COUNT(*)}; exemplars: the worker stream; else cells
        if tag:
            return lkcpu.evaluate_tag_counts(pr, tag, 10, blobs, threads, timing=timing)
        if exemplar:
            return lkcpu.evaluate_exemplar_rows(pr, 10, blobs, threads, timing=timing)
        return lkcpu.evaluate_cell_table(pr, 10, blobs, threads, timing=timing)

    def run():
        evaluate()   # warm (page-in, thread pool)
        log(f"rank {rank}: cpu baseline warm run done")   # (progress: a C5 shard takes ~45 s per run)
        times, table = [], None
        for i in range(3):
            t = []
            table = evaluate(timing=t)
            times.append(t[0])
            log(f"rank {rank}: cpu baseline run {i + 1}/3: {t[0]:.3f} s")
        return sorted(times)[1], table

    if concurrent:
        dt, table = run()
    else:   # ranks sharing one GPU's CPU share take turns, so each is timed on the full share
        for r in range(world):
            if r == rank:
                dt, table = run()
            dist.barrier()
    log(f"rank {rank}: cpu baseline {n} segments x {args.rows} rows in {dt:.3f}s (median of 3) on {threads} threads "
        f"({_cpu_model()}, {os.cpu_count()} CPUs visible)")
    full = n == len(segs)
    if world > 1:   # every rank's shard time and cells -> rank 0
        log(f"rank {rank}: sending the shard's cells to rank 0")
        times = [None] * world
        dist.all_gather_object(times, (dt, full))
        parts = [None] * world if rank == 0 else None
        dist.gather_object((table if tag or exemplar else table.to_dict()) if full else None, parts, dst=0)
        if rank != 0:
            return None, None
        full = all(f for _, f in times)
        dts = [t for t, _ in times]
        if full and tag:
            table = {}
            for p in parts:
                for k, c in p.items():
                    table[k] = table.get(k, 0) + c
        elif full and exemplar:   # query-api: the pods' streams merged (rank order) and take(limit)
            from oracle import exemplar as ex
            table = ex.merge_sorted_fold([[(t, v, k) for t, v, k, _ in p] for p in parts],
                                         pr.reverseSort)[:pr.baseExpr.limit]
        elif full:
            table = lkcpu.CellTable.concat([lkcpu.CellTable(**p) for p in parts])
    else:
        dts = [dt]
    validated = None
    if full:
        log(f"rank {rank}: comparing the GPU rows with the CPU restatement")
        has_gb = bool(q["group_bys"])
        want = (list(table),) if tag or exemplar else lkcpu.merge_cell_table(table, agg, has_gb)
        try:
            if exemplar:   # rows in stream order: timestamps, values (read, bit-exact), tag maps, glob (N = 1)
                got = list(zip(gpu_res.ts.tolist(), gpu_res.values.tolist(), gpu_res.tags, gpu_res.globs.tolist()))
                assert len(got) == len(table), f"{len(got)} rows vs {len(table)}"
                for i, (g, w) in enumerate(zip(got, table)):
                    assert g[0] == w[0] and g[1] == w[1], f"row {i}: (ts, value) {g[:2]} vs {w[:2]}"
                    assert g[2] == lkcpu.tags_of_key(w[2]), f"row {i}: tags {g[2]} vs {lkcpu.tags_of_key(w[2])}"
                    if world == 1:
                        assert g[3] == w[3], f"row {i}: glob {g[3]} vs {w[3]}"
            elif tag:   # the merged tag table: one row per tag text (NULL-like values together), value = COUNT(*)
                got = {}
                for v, t in zip(gpu_res.values.tolist(), gpu_res.tags):
                    k = t.get(tag)
                    assert int(t["count"]) == int(v), f"count tag {t['count']} vs value {v}"
                    assert k not in got, f"tag value {k!r} twice in the merged rows"
                    got[k] = int(v)
                assert got == table, f"tag counts differ: {sorted(set(got.items()) ^ set(table.items()))[:10]}"
            else:
                lkcpu.assert_columns_equal(result_columns(gpu_res), want, agg, "bench GPU rows vs CPU restatement")
            validated = {"ok": True, "rows": int(len(want[0])),
                         "against": "oracle/cpu (C++ restatement), full workload" +
                                    (f": {world} ranks' shard cells folded on rank 0 with query-api semantics"
                                     if world > 1 else "")}
        except AssertionError as e:
            validated = {"ok": False, "rows": int(len(want[0])), "error": str(e)[:500]}
        log(f"validation: {validated}")
    slowest = max(dts)
    rows_cpu = n * args.rows * world
    return ({"value": rows_cpu / slowest, "unit": "rows/s", "cores": threads * world, "kind": "port",
             "cpu_model": _cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": affinity,
             "core_limit": (f"OMP_NUM_THREADS={omp} per rank (the job's CPU share on this box; {affinity} CPUs in the "
                            f"affinity mask, {os.cpu_count()} on the host)") if omp else f"all {affinity} CPUs of the affinity mask",
             "per_rank_seconds": dts,
             "sample": (f"{n} of each rank's {len(segs)} segments ({rows_cpu} rows over {world} rank(s)), same query, "
                        f"oracle/cpu/lkcpu.cpp (C++17 + OpenMP restatement, {threads} threads per rank, median of 3 of "
                        f"the C++ evaluation)" +
                        (f"; ranks {'concurrently' if concurrent else 'one after another'}, value = all rows / the "
                         f"slowest rank's shard time" if world > 1 else ""))},
            validated)


if __name__ == "__main__":
    main()
