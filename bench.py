#!/usr/bin/env python3
"""Benchmark of the MI355X window/aggregate hot path (BASELINE.json metric, configs[1] = C2):

  SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo
  GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)       -- 1e8 synthetic events, 64 Ki keys, 1 MI355X

A step = one pass of the hot path over one batch: ek_reset + ek_push_batch of the 1e8-event batch
(inputs already resident in HBM) through the C ABI, which triggers 99 tumbling windows and writes their
GROUP BY result rows to HBM. Multi-GPU (torch.distributed.run): each rank owns a disjoint key-hash shard
of its own 1e8-event stream (weak scaling, no data-path collective); rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ekuiper-vioneta_amd"))

C2_SQL = ("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
          "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)")
N_EVENTS = 100_000_000
N_KEYS = 65536
EVENTS_PER_MS = 100
BYTES_IN_PER_EVENT = 4 + 8 + 8 + 8      # key u32, ts i64, temperature f64, humidity f64
BYTES_OUT_PER_ROW = 4 + 8 + 8 + 8       # key, avg, max, count
HBM_PEAK_GBS = 8000.0                   # MI355X_MICROARCH.md: 8.0 TB/s spec
PHASES = ("stats", "partition", "aggregate", "finalize")
KERNEL_OF_PHASE = {"stats": "k_stats", "partition": "k_part", "aggregate": "k_agg", "finalize": "k_finalize"}
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")


def _tmix(x):
    import torch
    x = x + torch.tensor(0x9E3779B97F4A7C15 - (1 << 64), dtype=torch.int64, device=x.device)
    x = x ^ ((x >> 30) & ((1 << 34) - 1))
    x = x * torch.tensor(0xBF58476D1CE4E5B9 - (1 << 64), dtype=torch.int64, device=x.device)
    x = x ^ ((x >> 27) & ((1 << 37) - 1))
    x = x * torch.tensor(0x94D049BB133111EB - (1 << 64), dtype=torch.int64, device=x.device)
    x = x ^ ((x >> 31) & ((1 << 33) - 1))
    return x


def make_device_stream(n, keys, dev, seed=44, key_offset=0, events_per_ms=EVENTS_PER_MS, t0=1541152480000):
    """ekgpu.synth.iot_stream generated directly in HBM (bit-identical counter-based splitmix64)."""
    import torch
    key = torch.empty(n, dtype=torch.int32, device=dev)
    ts = torch.empty(n, dtype=torch.int64, device=dev)
    temp = torch.empty(n, dtype=torch.float64, device=dev)
    hum = torch.empty(n, dtype=torch.float64, device=dev)
    base = seed << 40
    step = 1 << 24
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        i = torch.arange(lo, hi, dtype=torch.int64, device=dev)
        r0 = _tmix(base ^ (i * 8 + 0))
        hi1 = (r0 >> 1) & ((1 << 63) - 1)
        key[lo:hi] = (((hi1 % keys) * 2 + (r0 & 1)) % keys + key_offset).to(torch.int32)
        ts[lo:hi] = t0 + i // events_per_ms
        scale = 100.0 / 9007199254740992.0
        temp[lo:hi] = ((_tmix(base ^ (i * 8 + 1)) >> 11) & ((1 << 53) - 1)).to(torch.float64) * scale
        hum[lo:hi] = ((_tmix(base ^ (i * 8 + 2)) >> 11) & ((1 << 53) - 1)).to(torch.float64) * scale
    return [key, ts, temp, hum]


def cpu_baseline(sample_events):
    """The CPU oracle (C restatement of the reference per-tuple path, oracle/ekoracle.c) on the
    first `sample_events` events of the same stream: single thread (the reference runs a rule's window ->
    aggregate chain in one goroutine, operations.go:63-74), and as P key-hash shards on P host threads
    (reference semantics on all of this job's host cores)."""
    import threading
    import numpy as np
    from oracle import ekoracle
    from ekgpu.rule import compile_rule
    from ekgpu.synth import IOT_SCHEMA, iot_stream
    ekoracle.build()
    rule = compile_rule(C2_SQL, IOT_SCHEMA, num_keys=N_KEYS)
    key, ts, temp, hum = iot_stream(sample_events, N_KEYS, events_per_ms=EVENTS_PER_MS)
    t = time.perf_counter()
    run = ekoracle.run(rule.plan, [key, ts, temp, hum])
    dt = time.perf_counter() - t
    out = {"value": sample_events / dt, "unit": "events/s", "cores": 1, "kind": "port",
           "sample": f"first {sample_events} events of the C2 stream ({len(run.windows)} windows closed), "
                     f"oracle/ekoracle.c single-threaded, {dt:.1f} s"}
    # P key-hash shards (each a dense key space, like the GPU ranks), one thread each (ctypes drops the GIL)
    P = max(1, int(os.environ.get("EKGPU_CPU_THREADS", os.environ.get("OMP_NUM_THREADS", "8"))))
    shard = (key % P).astype(np.int64)
    parts = []
    for r in range(P):
        m = shard == r
        parts.append([(key[m] // P).astype(np.uint32), ts[m], temp[m], hum[m]])
    del shard
    prule = compile_rule(C2_SQL, IOT_SCHEMA, num_keys=(N_KEYS + P - 1) // P)
    errs = []

    def work(c):
        try:
            ekoracle.run(prule.plan, c)
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--events", type=int, default=N_EVENTS)
    ap.add_argument("--cpu-sample", type=int, default=int(os.environ.get("EKGPU_CPU_SAMPLE", N_EVENTS)))
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from ekgpu.engine import Engine
    from ekgpu.rule import compile_rule
    from ekgpu.synth import IOT_SCHEMA

    n = args.events
    # key-hash sharding: rank r owns a disjoint shard of the key space; the ingest side dictionary-encodes
    # the shard's keys densely (0..K-1), so every rank runs the same plan on its own stream
    rule = compile_rule(C2_SQL, IOT_SCHEMA, num_keys=N_KEYS)
    cols = make_device_stream(n, N_KEYS, dev, seed=44 + rank)
    torch.cuda.synchronize()
    eng = Engine(rule.plan, device=local)
    ptrs = [c.data_ptr() for c in cols]

    def step():
        eng.reset()
        eng.push_device(n, ptrs)

    for _ in range(args.warmup):
        step()
    # result sanity of the last warmup step (not timed)
    r = eng.poll_device()
    n_windows = int(r.n_windows)
    rows = sum(int(r.win_row_count[w]) for w in range(n_windows))
    eng.release(r)

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev_ms = 0.0
    ph_ms = [0.0] * 4
    ph_n = [0] * 4
    for _ in range(args.steps):
        step()
        st = eng.stats()
        dev_ms += st.last_batch_device_ms
        for k in range(4):
            ph_ms[k] += st.phase_ms[k]
            ph_n[k] += st.phase_launches[k]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt, dev_ms] + ph_ms, dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, dev_ms = float(t[0]), float(t[1])
        ph_ms = [float(x) for x in t[2:]]

    ms_per_step = dt * 1000.0 / args.steps
    value = n * world * args.steps / dt
    dev_ms_step = dev_ms / args.steps
    alg_bytes = n * BYTES_IN_PER_EVENT + rows * BYTES_OUT_PER_ROW
    path_gbs = alg_bytes / (dev_ms_step * 1e-3) / 1e9
    # dominant kernel: k_part (one launch per push here); its algorithmic bytes are the input columns
    # it must read once (28 B/event); staging writes are implementation traffic
    part_launch_ms = ph_ms[1] / max(1, ph_n[1])
    part_launches_per_step = ph_n[1] / args.steps
    part_alg = n * BYTES_IN_PER_EVENT / max(1.0, part_launches_per_step)
    achieved = part_alg / (part_launch_ms * 1e-3) / 1e9 if part_launch_ms > 0 else 0.0
    traffic, traffic_src = None, None
    if os.path.exists(PMC_SUMMARY):
        pm = json.load(open(PMC_SUMMARY))
        k = pm.get("kernels", {}).get("k_part")
        if k and k.get("events_per_launch") == n:
            traffic = k["hbm_bytes_per_launch"]
            traffic_src = os.path.relpath(PMC_SUMMARY, ROOT)
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
        "data": "synthetic (counter-based splitmix64 stream generated in HBM, SURVEY.md §8(d) C2 shape)",
        "config": {"workload": "C2: " + C2_SQL, "events_per_gpu": n, "keys_per_gpu": N_KEYS,
                   "event_rate": "100k ev/s event time (100 events per ms)", "windows_emitted": n_windows,
                   "rows_per_step": rows, "parallelism": f"key-hash shards x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "k_part (dominant kernel; HIP events around each launch on the engine stream)",
                     "algorithmic_bytes_per_launch": part_alg, "launch_ms": part_launch_ms,
                     "traffic_source": traffic_src,
                     "phase_ms_per_step": {PHASES[k]: ph_ms[k] / args.steps for k in range(4)},
                     "path": {"achieved": path_gbs, "frac": path_gbs / HBM_PEAK_GBS, "device_ms": dev_ms_step,
                              "algorithmic_bytes": alg_bytes,
                              "what": "whole ek_push_batch: 28 B/event in + 28 B/result row out over its device time"}},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_sample)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
