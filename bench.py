#!/usr/bin/env python3
"""Benchmark of the MI355X window/aggregate hot path (BASELINE.json metric; default config = configs[1] = C2):

  C2  SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo
      GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)           -- 1e8 synthetic events, 64 Ki keys per GPU

A step = one pass of the hot path over one batch (ek_reset + the batch's ek_push_batch through the C ABI, inputs
already resident in HBM); it triggers the batch's windows and writes their GROUP BY rows to HBM.
`--config C3|C4a|C4b|C5` runs the other BASELINE configs at their per-GPU sizes; `--config C1`
times the columnar JSON ingest + WHERE (messages/s).

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): ONE global stream of N x the per-GPU events
over N x the keys, key-hash sharded (mix64(key) % N, dense local ids per rank). Every rank runs its handle in
shard mode (ek_push_batch_global): the global WatermarkTuples of the (sorted) stream and the rows' global arrival
indices come from the router; sliding triggers (C4a) are exchanged with one all_gather over RCCL per step; C5's
un-grouped count(*) is merged with one all_gather. value = all ranks' events / the slowest rank's time (weak
scaling: per-GPU work fixed).

roofline: whole-step algorithmic bytes (one read of every referenced input column + one write of
the result rows) / ms_per_step against the 8 TB/s HBM peak; `kernels` splits the step per engine phase with the
HIP-event time of its launches on the engine stream and the algorithmic bytes that kernel itself must move.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ekuiper-vioneta_amd"))

HBM_PEAK_GBS = 8000.0                   # MI355X_MICROARCH.md: 8.0 TB/s spec
PHASES = ("stats", "partition", "aggregate", "finalize")
# the engine's phase clock (ek_stats.phase_ms, HIP events on the engine stream) per phase, and what runs in it
KERNEL_OF_PHASE = {"stats": "ts pass (k_stats, incl. a shared ek_batch_ts_stats) + pane bounds",
                   "partition": "partition (pane mode k_part | range mode key sort / MSD k_grp_hist+scatter)",
                   "aggregate": "aggregate (k_agg | k_small_win | key-major / grouping walk)",
                   "finalize": "finalize (k_finalize*)"}
T0 = 1541152480000

CONFIGS = {
    "C2": dict(sql="SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
                   "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)",
               n=100_000_000, keys=65536, epm=100, seed=44, t0=T0, in_cols=("key", "ts", "temperature", "humidity"),
               out_bytes=4 + 8 + 8 + 8),
    "C3": dict(sql="SELECT deviceId, sum(temperature), min(temperature), max(temperature) FROM demo "
                   "GROUP BY deviceId, HOPPINGWINDOW(ss, 60, 5)",
               n=25_000_000, keys=131072, epm=42, seed=91, t0=T0, in_cols=("key", "ts", "temperature"),
               out_bytes=4 + 3 * 8),
    "C4a": dict(sql="SELECT deviceId, stddev(temperature), var(temperature) FROM demo "
                    "GROUP BY deviceId, SLIDINGWINDOW(ss, 30) OVER (WHEN trig = 1) HAVING count(*) > 1",
                n=10_000_000, keys=1_000_000, epm=10, seed=92, t0=T0, in_cols=("key", "ts", "temperature", "trig"),
                out_bytes=4 + 8 + 8, trig=True),
    "C4b": dict(sql="SELECT deviceId, stddev(temperature), var(temperature) FROM demo "
                    "GROUP BY deviceId, COUNTWINDOW(1000) HAVING count(*) > 1",
                n=100_000_000, keys=1_000_000, epm=100, seed=93, t0=T0, in_cols=("key", "temperature"),
                out_bytes=4 + 8 + 8, processing_time=True, having_star_window=1000, having_star_col="temperature"),
    "C5": dict(sql="SELECT deviceId, median(temperature), percentile_cont(temperature, 0.9) FROM demo "
                   "GROUP BY deviceId, TUMBLINGWINDOW(ss, 60)",
               n=125_000_000, keys=12_500_000, epm=2084, seed=94, t0=1541152440000, in_cols=("key", "ts", "temperature"),
               out_bytes=4 + 8 + 8, sentinel=True, global_count="SELECT count(*) FROM demo GROUP BY TUMBLINGWINDOW(ss, 60)"),
}
COL_BYTES = {"key": 4, "ts": 8, "temperature": 8, "humidity": 8, "trig": 8}
# bytes each phase must move at least (per event / per result row)
PHASE_IN = {"stats": ("ts",), "partition": ("key", "temperature", "humidity", "trig")}

N_EVENTS = CONFIGS["C2"]["n"]
N_KEYS = CONFIGS["C2"]["keys"]
EVENTS_PER_MS = CONFIGS["C2"]["epm"]
C2_SQL = CONFIGS["C2"]["sql"]


def _tmix(x):
    import torch
    x = x + torch.tensor(0x9E3779B97F4A7C15 - (1 << 64), dtype=torch.int64, device=x.device)
    x = x ^ ((x >> 30) & ((1 << 34) - 1))
    x = x * torch.tensor(0xBF58476D1CE4E5B9 - (1 << 64), dtype=torch.int64, device=x.device)
    x = x ^ ((x >> 27) & ((1 << 37) - 1))
    x = x * torch.tensor(0x94D049BB133111EB - (1 << 64), dtype=torch.int64, device=x.device)
    x = x ^ ((x >> 31) & ((1 << 33) - 1))
    return x


def make_device_stream(n, keys, dev, seed=44, key_offset=0, events_per_ms=EVENTS_PER_MS, t0=T0, lo=0, hi=None):
    """ekgpu.synth.iot_stream generated directly in HBM (bit-identical counter-based splitmix64); rows [lo, hi)."""
    import torch
    hi = n if hi is None else hi
    m = hi - lo
    key = torch.empty(m, dtype=torch.int32, device=dev)
    ts = torch.empty(m, dtype=torch.int64, device=dev)
    temp = torch.empty(m, dtype=torch.float64, device=dev)
    hum = torch.empty(m, dtype=torch.float64, device=dev)
    base = seed << 40
    step = 1 << 24
    for a in range(lo, hi, step):
        b = min(hi, a + step)
        i = torch.arange(a, b, dtype=torch.int64, device=dev)
        r0 = _tmix(base ^ (i * 8 + 0))
        hi1 = (r0 >> 1) & ((1 << 63) - 1)
        key[a - lo:b - lo] = (((hi1 % keys) * 2 + (r0 & 1)) % keys + key_offset).to(torch.int32)
        ts[a - lo:b - lo] = t0 + i // events_per_ms
        scale = 100.0 / 9007199254740992.0
        temp[a - lo:b - lo] = ((_tmix(base ^ (i * 8 + 1)) >> 11) & ((1 << 53) - 1)).to(torch.float64) * scale
        hum[a - lo:b - lo] = ((_tmix(base ^ (i * 8 + 2)) >> 11) & ((1 << 53) - 1)).to(torch.float64) * scale
    return [key, ts, temp, hum]


def disorder_ts(ts, seed, ms):
    """`bench.py --disorder MS`: event i's ts moved back by a hash-chosen 0..MS ms, so the stream arrives out of
    order by at most MS ms (a rule with lateTolerance >= MS drops nothing)."""
    import torch
    i = torch.arange(len(ts), dtype=torch.int64, device=ts.device)
    return ts - (_tmix(i ^ (seed << 48)) & ((1 << 62) - 1)) % (ms + 1)


def trig_column(i):
    """C4a trigger flag of global event i: 1 in 1e4 events (tests/test_fullsize_parity_gpu.py)."""
    import torch
    return ((((i * 0x9E3779B1) >> 7) % 10_000) == 0).to(torch.int64)


def config_columns(cfg, cols, i=None):
    """The engine's columns for a config from the synthetic [key, ts, temperature, humidity] stream."""
    import torch
    key, ts, temp, hum = cols
    if cfg.get("trig"):
        return [key, ts, temp, hum, trig_column(i if i is not None else torch.arange(len(ts), device=ts.device))]
    return [key, ts, temp, hum]


def schema_of(cfg):
    from ekgpu.synth import IOT_SCHEMA
    return dict(IOT_SCHEMA, trig="bigint") if cfg.get("trig") else IOT_SCHEMA


def block_stream(cfg, world, rank, dev):
    """COUNTWINDOW rules shard by window blocks, not by key: window k is the arrivals [k n, (k + 1) n) of the
    global stream (window_op.go:390-418) and aggregates every key of that block only, so rank r takes the
    contiguous arrivals [r N, (r + 1) N) (N = per-GPU events, a multiple of n) and runs the single-GPU path on them:
    its windows are exactly the global windows r N / n ... (r + 1) N / n - 1 (no watermark, no exchange). Key-hash
    shards would cut every window into `world` pieces of n / world rows."""
    n_per = cfg["n"]
    c = make_device_stream(n_per * world, cfg["keys"] * world, dev, seed=cfg["seed"], events_per_ms=cfg["epm"] * world,
                           t0=cfg["t0"], lo=rank * n_per, hi=(rank + 1) * n_per)
    return config_columns(cfg, c), n_per * world, cfg["keys"] * world


def shard_stream(cfg, world, rank, dev):
    """Rank `rank`'s rows of the global stream (world x events, world x keys, world x rate): local columns with
    dense key ids, their global arrival indices, and the number of global events."""
    import torch
    n_glob, k_glob, epm = cfg["n"] * world, cfg["keys"] * world, cfg["epm"] * world
    parts, arrs = [], []
    step = 1 << 25
    for lo in range(0, n_glob, step):
        hi = min(n_glob, lo + step)
        c = make_device_stream(n_glob, k_glob, dev, seed=cfg["seed"], events_per_ms=epm, t0=cfg["t0"], lo=lo, hi=hi)
        i = torch.arange(lo, hi, dtype=torch.int64, device=dev)
        c = config_columns(cfg, c, i)
        own = (_tmix(c[0].to(torch.int64)) & ((1 << 62) - 1)) % world == rank
        parts.append([x[own] for x in c])
        arrs.append(i[own])
        del c, i, own
    cols = [torch.cat([p[k] for p in parts]) for k in range(len(parts[0]))]
    arr = torch.cat(arrs)
    del parts, arrs
    uniq, inv = torch.unique(cols[0], return_inverse=True)
    cols[0] = inv.to(torch.int32)
    return cols, arr, n_glob, int(uniq.numel())


def global_tuples(cfg, world, n_glob):
    """WatermarkTuples of the sorted synthetic global stream (lateTolerance 0): the stream max advances at every
    first event of a millisecond (ts = t0 + i // (epm * world))."""
    import numpy as np
    epm = cfg["epm"] * world
    wa = np.arange(0, n_glob, epm, dtype=np.int64)
    wt = cfg["t0"] + np.arange(len(wa), dtype=np.int64)
    return {"wm_arrival": wa, "wm_ts": wt, "arrivals_end": n_glob, "all_accepted": True, "max_wm_step": 1,
            "origin_known": True, "origin_ts": cfg["t0"], "origin_arrival": 0}


CPU_SAMPLE = {"C2": 100_000_000, "C3": 15_000_000, "C4a": 1_000_000, "C4b": 50_000_000, "C5": 30_000_000}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


PHASE_EVERY = int(os.environ.get("EKGPU_BENCH_PHASE_EVERY", "4"))   # timed steps per step with phase events


def committed_traffic(config, sim, events):
    """HBM bytes per step from the newest committed rocprofv3 PMC summary of this workload (tools/profile_configs.py);
    (None, None) when none matches its size."""
    for rnd in ("r06", "r05", "r04", "r03"):
        pmc = os.path.join(ROOT, "profiles", f"{rnd}_pmc_{config}{sim}.json")
        if not os.path.exists(pmc):
            continue
        pm = json.load(open(pmc))
        if pm.get("events_per_gpu") == events:
            return pm.get("hbm_bytes_per_step"), os.path.relpath(pmc, ROOT)
    return None, None


def cpu_baseline(name, cfg, sample_events):
    """The CPU oracle (C restatement of the reference per-tuple path, oracle/ekoracle.c) on the first
    `sample_events` events of the config's stream (the same synthetic generator, numpy side): single thread (the
    reference runs a rule's window -> aggregate chain in one goroutine, operations.go:63-74), and for rules that
    shard by key without changing their windows (tumbling / hopping GROUP BY key: C2, C3, C5) also as P key-hash
    shards on P host threads (reference semantics on all of this job's host cores). COUNTWINDOW
    blocks (C4b) and OVER (WHEN) triggers (C4a) are global over the stream, so those report one thread only."""
    import threading
    import numpy as np
    from oracle import ekoracle
    from ekgpu.rule import compile_rule
    from ekgpu.synth import iot_stream
    ekoracle.build()
    iet = not cfg.get("processing_time")
    keys = cfg["keys"]
    key, ts, temp, hum = iot_stream(sample_events, keys, seed=cfg["seed"], events_per_ms=cfg["epm"], t0=cfg["t0"])
    cols = [key, ts, temp, hum]
    if cfg.get("trig"):
        i = np.arange(sample_events, dtype=np.int64)
        cols.append(((((i * 0x9E3779B1) >> 7) % 10_000) == 0).astype(np.int64))
    if cfg.get("sentinel"):   # C5: the event at the window end that closes the one window
        end = cfg["t0"] + 60_000
        cols = [np.append(cols[0], np.uint32(0)), np.append(cols[1], np.int64(end)), np.append(cols[2], 50.0),
                np.append(cols[3], 50.0)]
    rules = [compile_rule(cfg["sql"], schema_of(cfg), num_keys=keys, is_event_time=iet)]
    if cfg.get("global_count"):
        rules.append(compile_rule(cfg["global_count"], schema_of(cfg), num_keys=1, is_event_time=iet))
    t = time.perf_counter()
    nwin = 0
    for r in rules:
        nwin += len(ekoracle.run(r.plan, cols).windows)
    dt = time.perf_counter() - t
    out = {"value": sample_events / dt, "unit": "events/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
           "sample": f"first {sample_events} events of the {name} stream ({nwin} windows closed), "
                     f"oracle/ekoracle.c single-threaded, {dt:.1f} s"}
    if cfg.get("trig") or cfg.get("processing_time"):
        return out
    P = max(1, int(os.environ.get("EKGPU_CPU_THREADS", os.environ.get("OMP_NUM_THREADS", "8"))))
    shard = (cols[0] % P).astype(np.int64)
    parts = []
    for r in range(P):
        m = shard == r
        parts.append([(cols[0][m] // P).astype(np.uint32)] + [c[m] for c in cols[1:]])
    del shard
    prules = [compile_rule(cfg["sql"], schema_of(cfg), num_keys=(keys + P - 1) // P, is_event_time=iet)]
    errs = []

    def work(c):
        try:
            for r in prules:
                ekoracle.run(r.plan, c)
            if cfg.get("global_count"):   # the shard's partial count(*); the P partials add up on the host
                ekoracle.run(rules[1].plan, c)
        except Exception as e:   # noqa: BLE001  (reported, not swallowed)
            errs.append(e)
    th = [threading.Thread(target=work, args=(c,)) for c in parts]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dtp = time.perf_counter() - t
    if errs:
        raise errs[0]
    out["parallel"] = {"value": sample_events / dtp, "unit": "events/s", "cores": P, "kind": "port",
                       "sample": f"the same events as {P} key-hash shards, one oracle instance per host thread, {dtp:.1f} s"}
    return out


def ingest_inclusive(eng, cols, n, steps=2, chunks=8):
    """C2 fed from host memory, reported beside `value` (never as it): the step's columns start in pinned host
    memory and the results end in host memory.
      serial:    one ek_push_batch of host columns (EK_MEM_HOST: the H2D copy inside the push), then ek_poll_results;
      pipelined: the batch cut into `chunks` micro-batches, each copied H2D on a side stream into one of two device
                 buffers while the engine aggregates the previous one (hipMemcpyAsync double buffering), then the poll."""
    import numpy as np
    import torch
    host = [c.cpu().pin_memory() for c in cols]
    arrs = [h.numpy() for h in host]
    in_bytes = sum(a.nbytes for a in arrs)

    def serial():
        eng.reset()
        eng.push_host(arrs)
        return sum(len(w.keys) for w in eng.poll())

    bounds = np.linspace(0, n, chunks + 1).astype(np.int64)
    csz = int(np.max(np.diff(bounds)))
    dbuf = [[torch.empty(csz, dtype=c.dtype, device=cols[0].device) for c in cols] for _ in range(2)]
    side = torch.cuda.Stream(device=cols[0].device)

    def issue(i):
        lo, hi = int(bounds[i]), int(bounds[i + 1])
        with torch.cuda.stream(side):
            for h, d in zip(host, dbuf[i % 2]):
                d[: hi - lo].copy_(h[lo:hi], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        return ev

    def pipelined():
        eng.reset()
        evs = {0: issue(0)}
        for i in range(chunks):
            if i + 1 < chunks:
                evs[i + 1] = issue(i + 1)     # its buffer's previous chunk (i - 1) was fully consumed below
            evs[i].synchronize()
            eng.push_device(int(bounds[i + 1] - bounds[i]), [d.data_ptr() for d in dbuf[i % 2]])
            eng.sync()
        return sum(len(w.keys) for w in eng.poll())

    out = {"h2d_bytes": in_bytes}
    for name, fn in (("serial", serial), ("pipelined", pipelined)):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        rows = 0
        for _ in range(steps):
            rows += fn()
        dt = (time.perf_counter() - t) / steps
        out[name] = {"events_per_s": n / dt, "ms_per_step": dt * 1e3, "rows_to_host": rows // steps}
    out["events_per_s"] = max(out["serial"]["events_per_s"], out["pipelined"]["events_per_s"])
    out["what"] = (f"pinned host columns -> device -> results polled to host; pipelined = {chunks} micro-batches, "
                   "H2D of the next overlapped with the aggregation of the current (two device buffers)")
    return out


def bench_c1(args):
    """C1: 1e6 schemaless JSON payloads {"temperature":T,"humidity":H}, T, H integers in [0, 100],
    decoded on the GPU (ek_json_decode: every number -> float64, converter.go:507-520) and filtered by
    SELECT * FROM demo WHERE temperature > 50 (ek_push_batch, window-less FilterOp). A step = decode + filter of the
    whole micro-batch with the payload bytes already in HBM; `host_fed` repeats it from pinned host memory (H2D
    included)."""
    import numpy as np
    import torch
    from ekgpu.engine import Engine, JsonDecoder
    from ekgpu.rule import compile_rule
    n = args.events or 1_000_000
    rng = np.random.default_rng(42 + 1)
    t = rng.integers(0, 101, n)
    h = rng.integers(0, 101, n)
    msgs = [f'{{"temperature":{a},"humidity":{b}}}'.encode() for a, b in zip(t.tolist(), h.tolist())]
    lens = np.fromiter((len(m) for m in msgs), dtype=np.int64, count=n)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    blob = np.frombuffer(b"".join(msgs), dtype=np.uint8)
    dev = torch.device("cuda", 0)
    d_blob = torch.from_numpy(blob.copy()).to(dev)
    d_offs = torch.from_numpy(offs).to(dev)
    dec = JsonDecoder.schemaless(["temperature", "humidity"])
    rule = compile_rule("SELECT * FROM demo WHERE temperature > 50", {"temperature": "float", "humidity": "float"},
                        is_event_time=False)
    eng = Engine(rule.plan, device=0)

    def step():
        b = dec.decode_device(d_blob.data_ptr(), len(blob), d_offs.data_ptr(), n)
        eng.reset()
        eng.push_batch(b)

    for _ in range(args.warmup):
        step()
    r = eng.poll_device()
    rows = int(r.win_row_count[0]) if int(r.n_windows) else 0
    eng.release(r)
    assert rows == int((t > 50).sum()), (rows, int((t > 50).sum()))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    # host-fed: payload bytes + offsets in pinned host memory, copied by ek_json_decode
    hb = torch.from_numpy(blob.copy()).pin_memory()
    ho = torch.from_numpy(offs).pin_memory()
    hb_np, ho_np = hb.numpy(), ho.numpy()
    dec.decode(hb_np, ho_np)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        b = dec.decode(hb_np, ho_np)
        eng.reset()
        eng.push_batch(b)
    eng.sync()
    dth = (time.perf_counter() - t1) / args.steps
    alg = len(blob) + 8 * (n + 1) + rows * (8 + 8 + 8)
    traffic, traffic_src = committed_traffic("C1", "", 0)   # the C1 PMC summary carries no event count (messages)
    out = {"metric": "messages/sec decoded and filtered (C1 JSON ingest + WHERE)", "value": n / dt, "unit": "messages/s",
           "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic (1e6 schemaless JSON payloads, integer T/H uniform in [0, 100], seed 43)",
           "config": {"workload": "C1: JSON decode + SELECT * FROM demo WHERE temperature > 50", "messages": n,
                      "payload_bytes": int(len(blob)), "rows_out": rows},
           "roofline": {"bound": "hbm", "achieved": alg / dt / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": alg / dt / 1e9 / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                        "what": "payload bytes + offsets read + passing rows x (row index + 2 f64 columns) written, over ms_per_step"},
           "host_fed": {"messages_per_s": n / dth, "ms_per_step": dth * 1e3,
                        "what": "payloads in pinned host memory: H2D inside ek_json_decode, then the filter"}}
    if not args.no_cpu:
        # CPU baseline: the same payloads decoded one message at a time (json.loads: every number float64, as the
        # schemaless converter.go:507-520) and filtered by WHERE temperature > 50 (filter_operator.go:36-90)
        t2 = time.perf_counter()
        kept = 0
        for m in msgs:
            d = json.loads(m)
            t_ = d.get("temperature")
            if t_ is not None and float(t_) > 50:
                kept += 1
        dtc = time.perf_counter() - t2
        assert kept == rows
        out["cpu_baseline"] = {"value": n / dtc, "unit": "messages/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
                               "sample": f"all {n} payloads, json.loads + WHERE per message (Python 3, C json decoder), {dtc:.1f} s"}
    print(json.dumps(out), flush=True)
    eng.close()
    dec.close()


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (one per GPU, RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run would) before this process touches a GPU, and
    exit with the first failing rank's code. Rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc != 0), 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS) + ["C1"])
    ap.add_argument("--events", type=int, default=0, help="override the per-GPU event count")
    ap.add_argument("--cpu-sample", type=int, default=int(os.environ.get("EKGPU_CPU_SAMPLE", "0")),
                    help="events of the CPU baseline sample (default: CPU_SAMPLE of the config, ~10 s single-threaded)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ingest", action="store_true")
    ap.add_argument("--no-shared-stats", action="store_true",
                    help="C5: each rule scans the source's timestamps itself (no ek_batch_ts_stats sharing)")
    ap.add_argument("--sim-world", type=int, default=0,
                    help="one process plays rank 0 of an N-GPU run in shard mode (no collective; a single-GPU check of "
                         "the shard path: C4a then sees only its own triggers)")
    ap.add_argument("--no-route", action="store_true",
                    help="N > 1: every rank starts from its own key-hash shard of the global stream, partitioned at "
                         "setup (the host-ingest model of SURVEY.md §8(e)); by default every rank ingests a contiguous "
                         "slice of the global stream and the step routes it (ek_route_partition + all_to_all)")
    ap.add_argument("--disorder", type=int, default=0, metavar="MS",
                    help="event-time configs: every ts moved back by a hash-chosen 0..MS ms (the stream arrives out of "
                         "order) and the rule compiled with lateTolerance = MS, so nothing is late and the engine's "
                         "unsorted path (watermark release, multi-tile partition) is the one timed")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} (one rank per GPU): refusing to run",
              file=sys.stderr, flush=True)
        return 2
    if env_world is None and args.gpus > 1:
        return spawn_ranks(args.gpus)
    if args.config == "C1":
        return bench_c1(args)

    import numpy as np
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if os.environ.get("EKGPU_BENCH_ONE_DEVICE"):   # rehearsal of the N-rank path on one GPU (with a gloo backend)
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("EKGPU_DIST_BACKEND", "nccl"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if args.sim_world > 1 and world == 1:
        world = args.sim_world

    from ekgpu.engine import Engine
    from ekgpu.rule import compile_rule
    from ekgpu.shard import device_watermark, make_ctx

    cfg = dict(CONFIGS[args.config])
    if args.events:
        cfg["n"] = args.events
    iet = not cfg.get("processing_time")
    if world == 1:
        c = make_device_stream(cfg["n"], cfg["keys"], dev, seed=cfg["seed"], events_per_ms=cfg["epm"], t0=cfg["t0"])
        cols = config_columns(cfg, c)
        del c
        if args.disorder > 0 and iet:
            cols[1] = disorder_ts(cols[1], cfg["seed"], args.disorder)
        arr, n_glob, k_local = None, cfg["n"], cfg["keys"]
    elif cfg.get("processing_time"):
        cols, n_glob, k_local = block_stream(cfg, world, rank, dev)
        arr = None
    elif args.no_route:
        cols, arr, n_glob, k_local = shard_stream(cfg, world, rank, dev)
    else:
        # the rank's ingest slice of the global stream (global keys, arrivals [rank n, (rank + 1) n)); the router in the
        # step sends every row to its key's owner (ekgpu.route); the shard dictionaries are the owners' dense key ids
        from ekgpu.route import owned_key_map
        n_per, k_glob = cfg["n"], cfg["keys"] * world
        n_glob = n_per * world
        c = make_device_stream(n_glob, k_glob, dev, seed=cfg["seed"], events_per_ms=cfg["epm"] * world, t0=cfg["t0"],
                               lo=rank * n_per, hi=(rank + 1) * n_per)
        ingest = config_columns(cfg, c, torch.arange(rank * n_per, (rank + 1) * n_per, dtype=torch.int64, device=dev))
        del c
        if args.disorder > 0 and iet:
            ingest[1] = disorder_ts(ingest[1], cfg["seed"] + rank, args.disorder)
        key_map, owned = owned_key_map(k_glob, world, dev)
        k_local = owned[rank]
        cols, arr = None, None
    routed = world > 1 and not cfg.get("processing_time") and not args.no_route
    blocks = world > 1 and bool(cfg.get("processing_time"))   # window-block shards: the single-GPU path per rank
    route_ms = [0.0, 0.0]   # routed steps: partition, exchange (host clock around the synchronous calls)

    def route():
        """The step's router: this rank's ingest slice -> its owned rows of every rank, in global arrival order."""
        from ekgpu.route import route_exchange, route_partition
        nonlocal cols, arr, n, ptrs, ts_dev
        ta = time.perf_counter()
        types = [3] + [1] * (len(ingest) - 1)   # key EK_COL_U32, then 8-byte columns
        outs, arr_o, cnts = route_partition(ingest, types, 0, world, key_map, rank * cfg["n"], local)
        tb = time.perf_counter()
        got = route_exchange(outs + [arr_o], cnts, dist)
        torch.cuda.synchronize()
        route_ms[0] += (tb - ta) * 1e3
        route_ms[1] += (time.perf_counter() - tb) * 1e3
        cols, arr = got[:-1], got[-1]
        n = int(cols[0].numel())
        ptrs = [x.data_ptr() for x in cols]
        ts_dev = cols[1]

    n = 0
    ptrs = []
    ts_dev = None
    if routed:
        route()
    n = int(cols[0].numel())
    rule = compile_rule(cfg["sql"], schema_of(cfg), num_keys=max(1, k_local), is_event_time=iet,
                        late_tolerance_ms=args.disorder if iet else 0)
    torch.cuda.synchronize()
    eng = Engine(rule.plan, device=local)
    ptrs = [x.data_ptr() for x in cols]
    sent_ptrs, cnt_eng = None, None
    if cfg.get("sentinel"):
        # one event at the window end closes C5's single window (its key is outside the compared groups)
        end = cfg["t0"] + 60_000
        sent = [torch.tensor([0], dtype=torch.int32, device=dev), torch.tensor([end], dtype=torch.int64, device=dev),
                torch.tensor([50.0], dtype=torch.float64, device=dev), torch.tensor([50.0], dtype=torch.float64, device=dev)]
        sent_ptrs = [x.data_ptr() for x in sent]
    if cfg.get("global_count"):
        crule = compile_rule(cfg["global_count"], schema_of(cfg), num_keys=1, is_event_time=iet)
        cnt_eng = Engine(crule.plan, device=local)
    if world == 1:
        # pushes return with their work queued (ek_set_async): the step's host work overlaps the previous step's device
        # tail; the inputs are static device buffers, and the timed loop ends with a device-wide synchronize
        eng.set_async(True)
        if cnt_eng is not None:
            cnt_eng.set_async(True)
    ctx = None
    if world > 1 and not blocks:
        tup = global_tuples(cfg, world, n_glob) if iet else {
            "wm_arrival": np.zeros(0, np.int64), "wm_ts": np.zeros(0, np.int64), "arrivals_end": n_glob,
            "origin_known": False, "origin_ts": 0, "origin_arrival": 0}
        ctx_rows = make_ctx(tup, np.zeros(0, np.int64))
        ctx_rows.row_arrival = arr.data_ptr()
        ctx_rows.memory = 1   # EK_MEM_DEVICE: the rows' arrivals live in HBM
        ctx = ctx_rows
        if cfg.get("sentinel"):
            sent_tup = {"wm_arrival": np.array([n_glob], np.int64), "wm_ts": np.array([cfg["t0"] + 60_000], np.int64),
                        "arrivals_end": n_glob + 1, "all_accepted": True, "max_wm_step": 0, "origin_known": True,
                        "origin_ts": cfg["t0"], "origin_arrival": 0}
            sent_ctx = make_ctx(sent_tup, np.zeros(0, np.int64))

    want_list = bool(cfg.get("trig") or cfg.get("sentinel"))   # range-mode windows take the full tuple list
    ts_dev = cols[1]

    # C5's second rule (the global count(*)) runs beside the grouped rule on a host thread of its own, as eKuiper runs
    # every rule in its own goroutines; each engine has its own HIP stream (ctypes releases the GIL in the calls)
    pool = None
    if cnt_eng is not None:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=1)

    # the two rules read one source batch: its timestamp statistics are computed once (ek_batch_ts_stats) and shared by
    # both pushes, as eKuiper's shared source feeds every subscribed rule (subtopo.go)
    share_stats = cnt_eng is not None and iet and not args.no_shared_stats
    shared = None

    def count_rule(c):
        cnt_eng.reset()
        if world == 1 or blocks:
            cnt_eng.push_device(n, ptrs, ts_stats=shared)
            if sent_ptrs:
                cnt_eng.push_device(1, sent_ptrs)
        else:
            cnt_eng.push_global_device(n, ptrs, c)
            if sent_ptrs:
                cnt_eng.push_global(None, sent_ctx)

    last_global = None
    count_pp = None
    if cnt_eng is not None:
        from ekgpu.dist import global_windows, make_partial_plan
        count_pp = make_partial_plan(crule)

    def step():
        nonlocal ctx, tup, shared, cols, arr, n, ptrs, ts_dev
        eng.reset()
        fut = None
        if world == 1 or blocks:
            if share_stats:
                shared = eng.batch_ts_stats(n, ptrs)   # inside the timed step
            if pool is not None:
                fut = pool.submit(count_rule, None)
            eng.push_device(n, ptrs, ts_stats=shared)
            if sent_ptrs:
                eng.push_device(1, sent_ptrs)
        else:
            if routed:
                route()   # the key-hash partition and the exchange, inside the timed step
            if iet and dist is not None:
                # the router (global WatermarkOp) runs inside the timed step, on the ranks' own rows
                tup = device_watermark(ts_dev, arr, args.disorder, dist, want_list)
                tup["arrivals_end"] = n_glob
                ctx = make_ctx(tup, np.zeros(0, np.int64))
                ctx.row_arrival = arr.data_ptr()
                ctx.memory = 1
            g = ctx
            if pool is not None:
                fut = pool.submit(count_rule, ctx)
            if cfg.get("trig"):
                from ekgpu.dist import exchange_triggers
                ta, tt = eng.shard_triggers_device(n, ptrs, g)
                ga, gt = exchange_triggers(ta, tt) if dist else (ta, tt)
                g = make_ctx(tup, np.zeros(0, np.int64), ga, gt)
                g.row_arrival = arr.data_ptr()
                g.memory = 1
            eng.push_global_device(n, ptrs, g)
            if sent_ptrs:
                eng.push_global(None, sent_ctx)
        if fut is not None:
            fut.result()   # both rules' pushes are inside the step
            if dist is not None and not blocks:
                # the reference's final result gather of the global (un-grouped) count(*): every rank's per-window
                # partial, one all_gather over RCCL, merged (ekgpu.dist.global_windows) — inside the timed step
                nonlocal last_global
                last_global = global_windows(count_pp, cnt_eng.poll())

    for _ in range(args.warmup):
        step()
    # result sanity of the last warmup step (not timed)
    r = eng.poll_device()
    n_windows = int(r.n_windows)
    rows = sum(int(r.win_row_count[w]) for w in range(n_windows))
    eng.release(r)
    global_count = None
    if cnt_eng is not None:
        if dist and not blocks:
            global_count = [w.values for w in last_global]
        else:
            cw = cnt_eng.poll()
            global_count = [int(w.values[0][0]) for w in cw if len(w.keys)]

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    st0 = eng.stats()   # running totals (the engine's pushes are asynchronous: read back after the loop)
    route_ms[0] = route_ms[1] = 0.0
    # per-kernel HIP-event timing is sampled: the engine records its phase events on one timed step in PHASE_EVERY
    # (ek_set_phase_timing; each event is a queue marker worth ~5-10 us of device idle per push), and the per-launch
    # averages come from those steps
    sampled = 0
    t0 = time.perf_counter()
    for i in range(args.steps):
        on = i % PHASE_EVERY == 0
        sampled += on
        eng.set_phase_timing(on)
        step()
    eng.set_phase_timing(True)
    # the engine's library links the system HIP runtime, torch its own: wait on the engines' streams themselves
    eng.sync()
    if cnt_eng is not None:
        cnt_eng.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    st1 = eng.stats()
    dev_ms = st1.device_ms_total - st0.device_ms_total
    ph_ms = [st1.phase_ms_total[k] - st0.phase_ms_total[k] for k in range(4)]
    ph_n = [st1.phase_launches_total[k] - st0.phase_launches_total[k] for k in range(4)]
    if dist:
        t = torch.tensor([dt, dev_ms] + ph_ms, dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, dev_ms = float(t[0]), float(t[1])
        ph_ms = [float(x) for x in t[2:]]

    ms_per_step = dt * 1000.0 / args.steps
    value = n_glob * args.steps / dt
    in_bytes_per_event = sum(COL_BYTES[c] for c in cfg["in_cols"])
    alg_bytes = n * in_bytes_per_event + rows * cfg["out_bytes"]
    formula_bytes = alg_bytes
    required = None
    if cfg.get("having_star_window"):
        # HAVING count(*) > 1 decides a group from its row count alone: the value column is only
        # needed for the rows of kept groups. The line counts what the step must move: every key + those values +
        # the result rows (the §8(d) formula, every referenced column of every event, is reported beside it)
        wl = cfg["having_star_window"]
        nwf = n // wl
        kk = cols[0][: nwf * wl].view(nwf, wl).to(torch.int64).sort(dim=1).values
        eq = kk[:, 1:] == kk[:, :-1]
        kept = torch.zeros_like(kk, dtype=torch.bool)
        kept[:, 1:] |= eq
        kept[:, :-1] |= eq
        kept_rows = int(kept.sum())
        del kk, eq, kept
        alg_bytes = n * COL_BYTES["key"] + kept_rows * COL_BYTES[cfg["having_star_col"]] + rows * cfg["out_bytes"]
        required = {"bytes_per_step": alg_bytes, "kept_group_rows": kept_rows,
                    "what": "every key (4 B) + the value column of the rows of groups HAVING count(*) > 1 keeps (8 B) "
                            "+ result rows; the rows of dropped one-row groups never need their value"}
    achieved = alg_bytes / (ms_per_step * 1e-3) / 1e9
    kernels = {}
    for k, ph in enumerate(PHASES):
        if ph_n[k] == 0:
            continue
        launch_ms = ph_ms[k] / ph_n[k]
        per_step = ph_n[k] / sampled
        if ph == "stats":
            kb = n * 8 if iet else 0
        elif ph == "partition":
            # (the fused sorted pass reads ts in the partition pass itself: no stats phase then)
            fused = iet and ph_n[PHASES.index("stats")] == 0
            kb = n * sum(COL_BYTES[c] for c in cfg["in_cols"] if c != "ts" or fused)
        elif ph_n[PHASES.index("partition")] == 0:
            # no partition pass (range windows: k_small_win / the key-major walks read the event columns
            # themselves): the aggregate kernels move the step's bytes less what the stats pass read
            kb = alg_bytes - (n * 8 if iet and ph_n[PHASES.index("stats")] else 0)
        else:
            kb = rows * cfg["out_bytes"]
        kb_launch = kb / per_step
        kernels[KERNEL_OF_PHASE[ph]] = {"launch_ms": launch_ms, "launches_per_step": per_step,
                                        "algorithmic_bytes_per_launch": kb_launch,
                                        "achieved_gbs": kb_launch / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else None}
    dominant = max(kernels.items(), key=lambda kv: kv[1]["launch_ms"] * kv[1]["launches_per_step"])[0] if kernels else None
    sim = f"_sim{world}" if args.sim_world > 1 else ""
    traffic, traffic_src = committed_traffic(args.config, sim, n) if (world == 1 or sim) else (None, None)
    out = {
        "metric": "events/sec (whole node) for windowed GROUP BY at 1/2/4/8 GPUs; % HBM peak",
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (counter-based splitmix64 stream generated in HBM, SURVEY.md §8(d) shape)",
        "config": {"workload": f"{args.config}: {cfg['sql']}", "events_per_gpu": cfg["n"], "keys_per_gpu": cfg["keys"],
                   "events_total": n_glob, "events_rank0": n, "windows_emitted": n_windows, "rows_per_step_rank0": rows,
                   "event_rate": f"{cfg['epm'] * world} events per ms of event time" if iet else "processing time",
                   "parallelism": f"window-block shards x{world} (COUNTWINDOW: contiguous global arrivals per rank)" if blocks else
                                  f"key-hash shards x{world}" + (" (shard mode: global WatermarkTuples, global arrivals"
                                                                  + (", trigger all_gather" if cfg.get("trig") else "")
                                                                  + (", count(*) all_gather" if cfg.get("global_count") else "")
                                                                  + ")" if world > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "what": (f"whole step: {in_bytes_per_event} B/event in + {cfg['out_bytes']} B/result row out "
                              f"(SURVEY.md §8(d)) over ms_per_step (driver clock)") if required is None else
                             "whole step: the bytes the step must move (required_bytes) over ms_per_step (driver clock)",
                     "algorithmic_bytes_per_step": alg_bytes, "device_ms_per_step": dev_ms / args.steps,
                     "formula_bytes_per_step": formula_bytes,
                     "formula_frac": formula_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "required_bytes": required,
                     "dominant_kernel": dominant, "kernels": kernels,
                     "kernel_timing": f"HIP events on the engine stream around each phase, recorded on {sampled} of the "
                                      f"{args.steps} timed steps (one in {PHASE_EVERY}); launch_ms = their average"},
    }
    out["config"]["fused_sorted_batches_last_step"] = int(st1.fused_batches)   # (stream counters restart at ek_reset)
    if routed:
        rt = torch.tensor(route_ms, dtype=torch.float64, device=dev)
        dist.all_reduce(rt, op=dist.ReduceOp.MAX)
        out["config"]["routing"] = {
            "partition_ms_per_step": float(rt[0]) / args.steps, "exchange_ms_per_step": float(rt[1]) / args.steps,
            "what": "inside the timed step, max over ranks: every rank ingests a contiguous slice of the global stream; "
                    "ek_route_partition splits it by owner = mix64(key) mod N (HIP, stable, keys renamed to the owner's "
                    "dense ids) and one all_to_all per column (RCCL) delivers every rank its rows in global arrival order"}
        out["config"]["parallelism"] += " (routed in the step: ek_route_partition + all_to_all)"
    if global_count is not None:
        out["config"]["global_count"] = str(global_count)[:200]
        out["config"]["shared_ts_stats"] = bool(share_stats)
    if args.disorder > 0 and iet:
        out["config"]["disorder_ms"] = args.disorder
        out["config"]["late_tolerance_ms"] = args.disorder
    if rank == 0 and world == 1 and args.config == "C2" and not args.no_ingest and not args.disorder:
        out["ingest_inclusive"] = ingest_inclusive(eng, cols, n)
    if rank == 0 and world == 1 and not args.no_cpu and not args.disorder:
        out["cpu_baseline"] = cpu_baseline(args.config, cfg, min(cfg["n"], args.cpu_sample or CPU_SAMPLE[args.config]))
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if cnt_eng is not None:
        cnt_eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
