"""Device probe: decode single messages and print the error code (debugging aid)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ekuiper-vioneta_amd"))
import torch
torch.cuda.init()
from ekgpu.engine import JsonDecoder
msgs = [b'{"e": "q\\"x"}', b'{"e": {"b": "q"}}', b'{"e": ["x}"]}', b'{"e": {"b": "q\\"x"}}', b'{"e": {"b": "}"}}',
        b'{"e": ["x"]}', b'{"e": [1, "x"]}', b'{"e": {"a": [1, "x}"]}}', b'{"e": {"a": 1, "b": "c"}}', b'{"e": {"a": "c"}}']
d = JsonDecoder({"id": "key", "ts": "bigint", "v": "float"})
for m in msgs:
    b = d.decode([m])
    print(b.n_rows, d.errors()[1], m)
