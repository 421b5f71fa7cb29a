#!/usr/bin/env python3
"""C2 engine-knob sweep on one GPU: the stream is generated once, one engine per setting (the knobs are read at
ek_create). Prints ms/step and per-phase device ms per setting. Usage: sweep_c2.py 'ENV=V,ENV2=V2' ['...' ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ekuiper-vioneta_amd"))

import torch  # noqa: E402
import bench  # noqa: E402
from ekgpu.engine import Engine  # noqa: E402
from ekgpu.rule import compile_rule  # noqa: E402


def main():
    cfg = bench.CONFIGS[os.environ.get("SWEEP_CONFIG", "C2")]
    dev = torch.device("cuda", 0)
    cols = bench.config_columns(cfg, bench.make_device_stream(cfg["n"], cfg["keys"], dev, seed=cfg["seed"],
                                                               events_per_ms=cfg["epm"], t0=cfg["t0"]))
    n = int(cols[0].numel())
    ptrs = [c.data_ptr() for c in cols]
    rule = compile_rule(cfg["sql"], bench.schema_of(cfg), num_keys=cfg["keys"], is_event_time=not cfg.get("processing_time"))
    steps = int(os.environ.get("SWEEP_STEPS", "10"))
    ref_rows = None
    for spec in sys.argv[1:] or [""]:
        saved = {}
        for kv in filter(None, spec.split(",")):
            k, v = kv.split("=")
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        eng = Engine(rule.plan, device=0)
        for _ in range(2):
            eng.reset()
            eng.push_device(n, ptrs)
        r = eng.poll_device()
        rows = sum(int(r.win_row_count[w]) for w in range(int(r.n_windows)))
        eng.release(r)
        torch.cuda.synchronize()
        ph = [0.0] * 4
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.reset()
            eng.push_device(n, ptrs)
            st = eng.stats()
            for k in range(4):
                ph[k] += st.phase_ms[k]
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3 / steps
        ref_rows = rows if ref_rows is None else ref_rows
        print(f"{spec or 'default':40s} ms/step {dt:7.3f}  phases(stats,part,agg,fin) "
              + " ".join(f"{x / steps:6.3f}" for x in ph) + f"  rows {rows}{'' if rows == ref_rows else ' MISMATCH'}",
              flush=True)
        eng.close()
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
