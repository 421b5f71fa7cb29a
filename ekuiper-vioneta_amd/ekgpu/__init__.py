"""ekgpu — MI355X-native window & aggregate engine for eKuiper rules (python side of the C ABI).

    from ekgpu.rule import compile_rule
    from ekgpu.engine import Engine
    rule = compile_rule("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
                        "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)", schema, num_keys=65536)
    eng = Engine(rule.plan)
    eng.push_host(columns)
    windows = eng.poll()
"""
from . import abi  # noqa: F401
from .rule import compile_rule  # noqa: F401
