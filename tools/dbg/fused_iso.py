"""Isolate a fused-pass mismatch: WHERE and / or a nullable column, fused vs EKGPU_FUSED=0, against the oracle."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "ekuiper-vioneta_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
torch.cuda.init()
from ekgpu import engine
from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from oracle import ekoracle
from parity import assert_windows_equal

cols = list(iot_stream(500_000, 2048, seed=44, events_per_ms=20))
rng = np.random.default_rng(7)
vh = (rng.random(500_000) > 0.1).astype(np.uint8)
for where in ("", "WHERE temperature > 20 "):
    for nullable in (False, True):
        for agg in ("max(humidity), count(humidity)", "max(humidity)", "count(humidity)"):
            sql = f"SELECT deviceId, avg(temperature), {agg} FROM demo {where}GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)"
            rule = compile_rule(sql, IOT_SCHEMA, num_keys=2048, debug_membership=True, nullable=("humidity",) if nullable else ())
            valid = [None, None, None, vh] if nullable else None
            exp = ekoracle.run(rule.plan, cols, valid)
            for fused in ("1", "0"):
                os.environ["EKGPU_FUSED"] = fused
                for batches in (1, 2):
                    eng = engine.Engine(rule.plan)
                    cuts = np.linspace(0, 500_000, batches + 1).astype(np.int64)
                    for b in range(batches):
                        lo, hi = cuts[b], cuts[b + 1]
                        eng.push_host([c[lo:hi] for c in cols], None if valid is None else [None if v is None else v[lo:hi] for v in valid])
                    got = eng.poll(); st = eng.stats(); eng.close()
                    try:
                        assert_windows_equal(rule.plan, got, exp.windows, check_members=True); r = "ok"
                    except AssertionError as e:
                        r = "FAIL " + str(e)[:160]
                    print(f"where={bool(where)} null={nullable} agg={agg!r} fused={fused} batches={batches} fz={st.fused_batches}: {r}", flush=True)
