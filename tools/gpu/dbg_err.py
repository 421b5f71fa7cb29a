"""Debug: window statuses / error texts of the error-text KAT rules, pane and range mode, 1 and 7 pushes."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "ekuiper-vioneta_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch
torch.cuda.init()
from ekgpu import engine as E
from ekgpu.rule import compile_rule
from oracle import ekoracle as O
import test_error_texts as T

for mode in ("pane", "range"):
    if mode == "range":
        os.environ["EKGPU_FORCE_RANGE"] = "1"
    for name, sql, texts in T.CASES:
        rule = compile_rule(sql, T.SCHEMA, num_keys=4)
        cols = T._cols()
        exp = O.run(rule.plan, cols)
        for nb in (1, 7):
            eng = E.Engine(rule.plan)
            for b in range(nb):
                lo, hi = b * len(cols[0]) // nb, (b + 1) * len(cols[0]) // nb
                eng.push_host([c[lo:hi] for c in cols])
            got = eng.poll()
            eng.close()
            g = [(w.start, w.end, w.status, w.error) for w in got]
            e = [(w.start, w.end, w.status, t) for w, t in zip(exp.windows, exp.errors)]
            print(mode, name, nb, "OK" if g == e else f"MISMATCH\n  got {g}\n  exp {e}", flush=True)
