"""One process per GPU, collectives over RCCL (torch.distributed "nccl").

The island model needs only small collectives: an all-gather of fixed-size
elite records every K generations (migration) and a max all-reduce (global
best / early stop / max-over-ranks timing).  On MI355X these run over RCCL on
the xGMI links; at these message sizes (a few KB to ~200 KB) they are
latency-bound, so we send one padded tensor per migration rather than many
small ones.  Without GPUs (tests, CPU hosts) the same API runs on gloo.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: Optional[object] = None   # torch.device used for collective buffers

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        """Several ranks (the island search's multi-rank semantics)."""
        return self.world_size > 1

    @property
    def group(self) -> bool:
        """A process group exists: the collective helpers go through it (RCCL /
        gloo) -- also for a one-rank group (FKS_DIST_GROUP=1), which exercises
        the collective path on a single GPU with results equal to the local one."""
        return self.backend != "none"


_ctx: Optional[DistContext] = None


def init_distributed(backend: Optional[str] = None, use_gpu: Optional[bool] = None,
                     force_group: Optional[bool] = None) -> DistContext:
    """Initialise from torchrun-style env vars (RANK/WORLD_SIZE/LOCAL_RANK,
    MASTER_ADDR defaults to 127.0.0.1).  Single-process runs need nothing,
    unless `force_group` (or FKS_DIST_GROUP=1) asks for a one-rank group."""
    global _ctx
    if _ctx is not None:
        return _ctx
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if force_group is None:
        force_group = os.environ.get("FKS_DIST_GROUP", "0") == "1"
    if world <= 1 and not force_group:
        _ctx = DistContext(rank=0, world_size=1, local_rank=local, backend="none")
        return _ctx
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    if backend is None:
        # FKS_DIST_BACKEND=gloo rehearses multi-rank GPU runs on a single-GPU box
        backend = os.environ.get("FKS_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    device = torch.device("cpu")
    if backend == "nccl":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    if not dist.is_initialized():
        import datetime
        kw = {}
        if os.environ.get("FKS_DIST_TIMEOUT_S"):
            # failure detection: a collective whose peer is gone raises after this long
            kw["timeout"] = datetime.timedelta(seconds=float(os.environ["FKS_DIST_TIMEOUT_S"]))
        attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT")
        if attempt is not None:
            # Under torchrun the agent's TCPStore outlives a restart round (same
            # MASTER_PORT), so a restarted group would read the previous round's
            # gloo / RCCL peer addresses from it and connect to dead sockets
            # ("connectFullMesh ... Connection refused").  Every round gets its
            # own key space instead.
            store, _, _ = next(dist.rendezvous("env://", rank=rank, world_size=world,
                                               timeout=kw.get("timeout", datetime.timedelta(minutes=10))))
            store = dist.PrefixStore(f"/fks/attempt_{attempt}", store)
            dist.init_process_group(backend=backend, store=store, rank=rank, world_size=world, **kw)
        else:
            dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    _ctx = DistContext(rank=rank, world_size=world, local_rank=local, backend=backend, device=device)
    return _ctx


_host_pg = None            # gloo group beside an RCCL default group (use_host_collectives)
_host_transport = False   # route the host-array collectives through it


def use_host_collectives(on: bool = True) -> bool:
    """Send the host-array collectives (all_gather_array[_async],
    all_reduce_max/sum, all_gather_bytes, barrier) over a gloo group beside
    RCCL (opened by the first such call: with the resident program grid on the
    device, RCCL collectives -- default or side stream -- wait for the grid to
    end, measured by tools/grid_coexist_probe.py).  Every rank must make the same call at
    the same point (it changes which group the next collective uses): the
    island search does it at construction when its configuration runs the
    resident program service.  Returns whether host collectives are now in use
    (False without an RCCL group: gloo-only and local runs are host already)."""
    global _host_transport, _host_pg
    ctx = context()
    hg = os.environ.get("FKS_HOST_GROUP", "1")
    if on and _host_pg is None and ctx.group and (
            (ctx.backend == "nccl" and hg != "0") or hg == "force"):   # force: a CPU (gloo-on-gloo) rehearsal
        # opened here, not in init_distributed: only runs that need it (the
        # service configurations) pay for a second group -- every rank reaches
        # this call at the same point, as new_group requires
        import torch.distributed as dist
        _host_pg = dist.new_group(backend="gloo")
    _host_transport = bool(on) and _host_pg is not None
    return _host_transport


def _host_group():
    """(group, device) of the next host-array collective."""
    ctx = context()
    if _host_transport and _host_pg is not None:
        import torch
        return _host_pg, torch.device("cpu")
    return None, ctx.device


def context() -> DistContext:
    return _ctx or init_distributed()


def barrier() -> None:
    ctx = context()
    if ctx.group:
        import torch.distributed as dist
        grp, _ = _host_group()
        if grp is not None:
            dist.barrier(group=grp)
        elif ctx.backend == "nccl":
            import torch
            dist.barrier(device_ids=[ctx.local_rank])
            torch.cuda.synchronize()
        else:
            dist.barrier()


def all_gather_array(x: np.ndarray) -> np.ndarray:
    """[world, *x.shape]: every rank's array (same shape/dtype on all ranks)."""
    ctx = context()
    if not ctx.group:
        return x[None].copy()
    import torch
    import torch.distributed as dist
    grp, d = _host_group()
    t = torch.from_numpy(np.ascontiguousarray(x)).to(d)
    out = [torch.empty_like(t) for _ in range(ctx.world_size)]
    dist.all_gather(out, t, group=grp)
    return np.stack([o.cpu().numpy() for o in out])


class PendingGather:
    """Handle of a non-blocking all-gather; `wait()` -> [world, *shape]."""

    def __init__(self, work=None, out=None, ready: Optional[np.ndarray] = None):
        self._work, self._out, self._ready = work, out, ready

    def done(self) -> bool:
        return self._ready is not None or self._work.is_completed()

    def wait(self) -> np.ndarray:
        if self._ready is None:
            self._work.wait()
            self._ready = np.stack([o.cpu().numpy() for o in self._out])
        return self._ready


def all_gather_array_async(x: np.ndarray) -> PendingGather:
    """Start an all-gather and return at once (RCCL runs it on its own stream
    while the caller keeps the GPU busy); the result is read with `.wait()`."""
    ctx = context()
    if not ctx.group:
        return PendingGather(ready=x[None].copy())
    import torch
    import torch.distributed as dist
    grp, d = _host_group()
    t = torch.from_numpy(np.ascontiguousarray(x)).to(d)
    out = [torch.empty_like(t) for _ in range(ctx.world_size)]
    work = dist.all_gather(out, t, async_op=True, group=grp)
    return PendingGather(work, out)


def all_reduce_max(v: float) -> float:
    ctx = context()
    if not ctx.group:
        return float(v)
    import torch
    import torch.distributed as dist
    grp, d = _host_group()
    t = torch.tensor([float(v)], dtype=torch.float64, device=d)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=grp)
    return float(t.item())


def all_reduce_sum(v: float) -> float:
    ctx = context()
    if not ctx.group:
        return float(v)
    import torch
    import torch.distributed as dist
    grp, d = _host_group()
    t = torch.tensor([float(v)], dtype=torch.float64, device=d)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=grp)
    return float(t.item())


def degrade_to_local(reason: str = "") -> DistContext:
    """Leave the process group after a failed collective and carry on as a
    single-rank job (every collective helper then runs locally).  The rank id
    is kept so this survivor keeps writing its own checkpoint file.  Used by
    the island search so that losing one rank does not end the run (SURVEY
    §5.3); the lost islands come back through `--resume` (see
    `IslandFunSearch.load_elastic`)."""
    global _ctx, _host_pg, _host_transport
    ctx = context()
    if ctx.group:
        import torch.distributed as dist
        try:
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:       # the group may already be broken; nothing left to release
            pass
    _host_pg, _host_transport = None, False
    _ctx = DistContext(rank=ctx.rank, world_size=1, local_rank=ctx.local_rank, backend="none",
                       device=ctx.device)
    return _ctx


def shutdown() -> None:
    global _ctx, _host_pg, _host_transport
    _host_pg, _host_transport = None, False
    if _ctx is not None and _ctx.group:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    _ctx = None


def all_gather_bytes(payload: bytes):
    """Every rank's byte string, whatever its length: one all-gather of the
    lengths, then one of the payloads padded to the longest (two small
    collectives; used where a record must never be truncated, e.g. the
    final cross-rank champion)."""
    ctx = context()
    if not ctx.group:
        return [bytes(payload)]
    n = all_gather_array(np.array([len(payload)], dtype=np.int64)).reshape(-1)
    buf = np.zeros(max(1, int(n.max())), dtype=np.uint8)
    buf[:len(payload)] = np.frombuffer(payload, dtype=np.uint8)
    allb = all_gather_array(buf)
    return [allb[r, :int(n[r])].tobytes() for r in range(ctx.world_size)]


# -------------------------------------------------------------------- program records
RECORD_BYTES = 4096   # fixed-width records (pack_programs): single programs, tests


class RecordTooLong(ValueError):
    """A program does not fit a fixed-width record (never sent truncated or empty)."""


def pack_programs(codes, scores, width: int = RECORD_BYTES) -> np.ndarray:
    """Fixed-size byte records [E, 16 + width]: score (f64), length (i64), utf-8 text.
    Raises `RecordTooLong` rather than emitting an empty slot; variable-length
    payloads go through `all_gather_bytes` / `pack_migrants`."""
    out = np.zeros((len(codes), 16 + width), dtype=np.uint8)
    for i, (c, s) in enumerate(zip(codes, scores)):
        b = c.encode("utf-8")
        if len(b) > width:
            raise RecordTooLong(f"program {i} is {len(b)} bytes, record width {width}")
        out[i, :8] = np.frombuffer(np.float64(s).tobytes(), dtype=np.uint8)
        out[i, 8:16] = np.frombuffer(np.int64(len(b)).tobytes(), dtype=np.uint8)
        out[i, 16:16 + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return out


def unpack_programs(rec: np.ndarray):
    res = []
    for row in rec.reshape(-1, rec.shape[-1]):
        n = int(np.frombuffer(row[8:16].tobytes(), dtype=np.int64)[0])
        if n <= 0:
            continue
        score = float(np.frombuffer(row[:8].tobytes(), dtype=np.float64)[0])
        res.append((bytes(row[16:16 + n]).decode("utf-8"), score))
    return res


# -------------------------------------------------------------------- migrant blobs
#: bytes per rank in a migration all-gather.  A rank's migrants travel as one
#: length-prefixed, zlib-compressed JSON blob; programs that follow the policy
#: template ship only their LLM body (a 3 KB program is ~0.4 KB on the wire), so
#: ~100+ migrants of any length fit.  One fixed size keeps the collective a
#: single (async-capable) all-gather; the links are latency-bound at this size.
MIGRANT_BLOB_BYTES = 1 << 18


def _template_parts():
    from ..policy.template import PolicyTemplate
    marker = "\x00BODY\x00"
    filled = PolicyTemplate.fill_template(marker)
    pre, post = filled.split(marker)
    return pre, post


def program_body(code: str):
    """(body, True) when `code` is the policy template around an LLM body,
    else (code, False)."""
    from ..policy.template import PolicyTemplate
    pre, post = _template_parts()
    if code.startswith(pre) and code.endswith(post) and len(code) >= len(pre) + len(post):
        body = code[len(pre):len(code) - len(post)]
        if PolicyTemplate.fill_template(body) == code:
            return body, True
    return code, False


def pack_migrants(records, capacity: int = MIGRANT_BLOB_BYTES, log=None) -> np.ndarray:
    """records: [(island, code, score)] best first -> uint8[capacity] blob.
    If the compressed blob does not fit, the lowest-scoring records are left
    out (each one logged through `log(dict)`) until it does."""
    import json
    import zlib
    items = []
    for isl, code, score in records:
        body, templ = program_body(code)
        items.append({"i": int(isl), "s": float(score), "t": int(templ), "c": body})
    dropped = 0
    while True:
        raw = zlib.compress(json.dumps(items).encode("utf-8"), 6)
        if len(raw) + 8 <= capacity or not items:
            break
        gone = items.pop()
        dropped += 1
        if log is not None:
            log(dict(kind="migrant_dropped", island=gone["i"], score=gone["s"], bytes=len(gone["c"]),
                     reason="migration blob full"))
    out = np.zeros(capacity, dtype=np.uint8)
    out[:8] = np.frombuffer(np.int64(len(raw)).tobytes(), dtype=np.uint8)
    out[8:8 + len(raw)] = np.frombuffer(raw, dtype=np.uint8)
    return out


def unpack_migrants(blob: np.ndarray):
    """[(island, code, score)] of one rank's blob."""
    import json
    import zlib
    from ..policy.template import PolicyTemplate
    b = np.ascontiguousarray(blob, dtype=np.uint8)
    n = int(np.frombuffer(b[:8].tobytes(), dtype=np.int64)[0])
    if n <= 0:
        return []
    items = json.loads(zlib.decompress(b[8:8 + n].tobytes()).decode("utf-8"))
    return [(it["i"], PolicyTemplate.fill_template(it["c"]) if it["t"] else it["c"], it["s"]) for it in items]
