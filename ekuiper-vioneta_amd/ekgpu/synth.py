"""Deterministic synthetic event streams; counter-based so any slice can be
generated independently: value(i, stream) = mix64((seed << 40) ^ (8*i + stream)).

C2 shape: deviceId u32 uniform over num_keys, ts = t0 + i // events_per_ms (ms), temperature and
humidity f64 uniform in [0, 100).
"""
import numpy as np

T0 = 1541152480000  # a 10 s boundary (second-of-minute 40)

_C1 = np.uint64(0x9E3779B97F4A7C15)
_C2 = np.uint64(0xBF58476D1CE4E5B9)
_C3 = np.uint64(0x94D049BB133111EB)


def mix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x += _C1
        x ^= x >> np.uint64(30)
        x *= _C2
        x ^= x >> np.uint64(27)
        x *= _C3
        x ^= x >> np.uint64(31)
    return x


def rand_u64(seed: int, lo: int, hi: int, stream: int) -> np.ndarray:
    i = np.arange(lo, hi, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) << np.uint64(40)) ^ (i * np.uint64(8) + np.uint64(stream))
    return mix64(x)


def uniform01(seed: int, lo: int, hi: int, stream: int) -> np.ndarray:
    return (rand_u64(seed, lo, hi, stream) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def iot_stream(n: int, num_keys: int, seed: int = 44, events_per_ms: int = 100, t0: int = T0, lo: int = 0):
    """Columns (deviceId u32, ts i64, temperature f64, humidity f64) for events [lo, lo+n)."""
    hi = lo + n
    key = (rand_u64(seed, lo, hi, 0) % np.uint64(num_keys)).astype(np.uint32)
    ts = t0 + np.arange(lo, hi, dtype=np.int64) // events_per_ms
    temp = uniform01(seed, lo, hi, 1) * 100.0
    hum = uniform01(seed, lo, hi, 2) * 100.0
    return key, ts, temp, hum


IOT_SCHEMA = {"deviceId": "key", "ts": "bigint", "temperature": "float", "humidity": "float"}
