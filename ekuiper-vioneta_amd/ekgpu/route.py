"""The key-hash router of a multi-GPU rule (gpu = hash(key) mod G per micro-batch), on the devices.

Every rank ingests a contiguous slice of the global stream. Per micro-batch the router
  1. splits the slice by owner rank (ek_route_partition, a HIP kernel: stable per-destination segments, each key renamed
     to its owner's dense id through the shard dictionary, each row's global arrival index materialised), and
  2. exchanges the segments with one all_to_all per column over the default process group (RCCL over xGMI for
     "nccl"; a gloo rehearsal group moves them through host memory).
A rank receives its rows in source-rank order, which is global arrival order (the slices are contiguous and ranked),
as ek_push_batch_global requires. The watermark over the whole stream is then ekgpu.shard.device_watermark.

The owner function is ek_mix64(key) & (2^62 - 1) mod G (include/ekgpu.h), the same as bench.py's synthetic shards.
"""
import ctypes as C
from typing import List, Sequence, Tuple

from . import abi as A
from .engine import EngineError, lib

_MASK62 = (1 << 62) - 1


def _bind():
    L = lib()
    if not getattr(L, "_route_bound", False):
        L.ek_route_partition.argtypes = [C.c_int, C.c_void_p, C.POINTER(A.ek_batch), C.POINTER(C.c_int32), C.c_int32,
                                         C.c_int32, C.c_void_p, C.c_uint32, C.c_int64, C.POINTER(C.c_void_p), C.c_void_p,
                                         C.POINTER(C.c_int64)]
        L.ek_route_partition.restype = C.c_int
        L._route_bound = True
    return L


def mix64_torch(x):
    """ek_mix64 on an int64 torch tensor (two's-complement wrap, logical shifts)."""
    import torch
    x = x + torch.tensor(0x9E3779B97F4A7C15 - (1 << 64), dtype=torch.int64, device=x.device)
    x = x ^ ((x >> 30) & ((1 << 34) - 1))
    x = x * torch.tensor(0xBF58476D1CE4E5B9 - (1 << 64), dtype=torch.int64, device=x.device)
    x = x ^ ((x >> 27) & ((1 << 37) - 1))
    x = x * torch.tensor(0x94D049BB133111EB - (1 << 64), dtype=torch.int64, device=x.device)
    x = x ^ ((x >> 31) & ((1 << 33) - 1))
    return x


def key_owner(keys, world: int):
    """Owner rank of every global key (torch tensor of any integer type)."""
    import torch
    return (mix64_torch(keys.to(torch.int64)) & _MASK62) % world


def owned_key_map(num_keys: int, world: int, device) -> Tuple["object", List[int]]:
    """The shard dictionaries of a dense global key space 0..num_keys-1: a device table global key -> dense id among
    its owner's keys (in key order), and every rank's key count."""
    import torch
    g = torch.arange(num_keys, dtype=torch.int64, device=device)
    own = key_owner(g, world)
    lut = torch.empty(num_keys, dtype=torch.int32, device=device)
    counts = []
    for r in range(world):
        m = own == r
        c = int(m.sum())
        lut[m] = torch.arange(c, dtype=torch.int32, device=device)
        counts.append(c)
    return lut, counts


def route_partition(cols: Sequence, col_types: Sequence[int], key_col: int, world: int, key_map, arrival_base: int,
                    device: int = 0):
    """One rank's ingest slice (device torch tensors, arrival order) -> (the same columns regrouped into `world`
    destination segments with owner-local keys, the rows' global arrivals, per-destination row counts)."""
    import torch
    L = _bind()
    n = int(cols[0].numel())
    outs = [torch.empty_like(c) for c in cols]
    arr = torch.empty(n, dtype=torch.int64, device=cols[0].device)
    b = A.ek_batch()
    b.n_rows = n
    b.memory = A.EK_MEM_DEVICE
    for k, c in enumerate(cols):
        b.columns[k] = c.data_ptr()
    ct = (C.c_int32 * A.EK_MAX_COLUMNS)(*list(col_types))
    op = (C.c_void_p * len(outs))(*[o.data_ptr() for o in outs])
    cnt = (C.c_int64 * world)()
    torch.cuda.synchronize(cols[0].device)   # the inputs are written by torch's runtime; the router runs on libekgpu's
    rc = L.ek_route_partition(device, None, C.byref(b), ct, key_col, world, key_map.data_ptr() if key_map is not None else None,
                              int(key_map.numel()) if key_map is not None else 0, arrival_base, op, arr.data_ptr(), cnt)
    if rc != 0:
        raise EngineError(rc, "ek_route_partition failed")
    return outs, arr, [int(x) for x in cnt]


def route_exchange(cols: Sequence, counts: Sequence[int], dist, group=None):
    """all_to_all of every column's destination segments: this rank's rows from every rank, in source-rank order."""
    import torch
    world = dist.get_world_size(group)
    dev = cols[0].device
    on_gpu = dist.get_backend(group) == "nccl"
    xdev = dev if on_gpu else torch.device("cpu")
    send = torch.tensor(list(counts), dtype=torch.int64, device=xdev)
    recv = torch.empty(world, dtype=torch.int64, device=xdev)
    dist.all_to_all_single(recv, send, group=group)
    rc = [int(x) for x in recv.tolist()]
    out = []
    for c in cols:
        src = c if on_gpu else c.cpu()
        dst = torch.empty(sum(rc), dtype=c.dtype, device=xdev)
        dist.all_to_all_single(dst, src, output_split_sizes=rc, input_split_sizes=list(counts), group=group)
        out.append(dst if on_gpu else dst.to(dev))
    return out
