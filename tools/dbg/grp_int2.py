import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ekuiper-vioneta_amd")); sys.path.insert(0, ROOT)
from ekgpu.rule import compile_rule
from ekgpu.engine import Engine
keys = 150_000
n = 80_000
rng = np.random.default_rng(1)
T0 = 1541152480000
k = rng.integers(0, 3000, n).astype(np.uint32)
ts = (T0 + np.arange(n) // 40).astype(np.int64)
v = rng.integers(-1000, 1000, n).astype(np.int64)
cut = int(np.searchsorted(ts, T0 + 1000))
for typ, col in (("bigint", v), ("float", v.astype(np.float64))):
    schema = {"k": "key", "ts": "bigint", "v": typ}
    rule = compile_rule("SELECT k, median(v), count(*), min(v), max(v) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)", schema, num_keys=keys)
    os.environ["EKGPU_GRP"] = "1"
    os.environ["EKGPU_KEYMAJOR"] = "1"
    eng = Engine(rule.plan)
    cols = [k, ts, col]
    eng.push_host([c[:cut] for c in cols]); eng.push_host([c[cut:] for c in cols])
    g = eng.poll()[0]; eng.close()
    bad = 0
    for i, key in enumerate(g.keys[:3000]):
        vals = np.sort(v[:cut][k[:cut] == key])
        cnt = int(g.values[1][i]); mn = g.values[2][i]; mx = g.values[3][i]
        if typ == "float":
            mn = np.int64(mn).view(np.float64); mx = np.int64(mx).view(np.float64)
        if cnt != len(vals) or mn != vals[0] or mx != vals[-1]:
            bad += 1
            if bad < 4: print(typ, "key", key, "cnt", cnt, len(vals), "min", mn, vals[0], "max", mx, vals[-1], "tag", g.tags[0][i], "med", g.values[0][i], vals)
    print(typ, "rows", len(g.keys), "bad(count/min/max)", bad)
    badm = 0
    for i, key in enumerate(g.keys[:3000]):
        vals = v[:cut][k[:cut] == key]
        sv = np.sort(vals)
        n2 = len(sv)
        exp_med = sv[n2 // 2] if n2 % 2 else (sv[n2 // 2 - 1] + sv[n2 // 2]) / 2
        t = int(g.tags[0][i]); raw = int(g.values[0][i])
        got = raw if t == 1 else float(np.int64(raw).view(np.float64))
        if got != exp_med:
            badm += 1
            if badm < 4: print(typ, "MED key", key, "n", n2, "got", t, got, "exp", exp_med, "arrival-order", list(vals), "sorted", list(sv))
    print(typ, "bad medians", badm)
