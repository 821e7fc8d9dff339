"""Process-group setup and the small collectives of the summarizer.

One process per GPU (``torchrun --nproc-per-node N``).  On ROCm the
``"nccl"`` backend of ``torch.distributed`` *is* RCCL, whose rings run over
the point-to-point xGMI links of the node; ``gloo`` is used on CPU-only hosts
(tests).  Rendezvous uses the ``MASTER_ADDR``/``MASTER_PORT`` env vars
(always 127.0.0.1 in this project's launchers).

Layout: ``world = dp * tp`` with tensor-parallel groups of consecutive ranks
(``[0..tp-1], [tp..2tp-1], ...``) so a TP group shares the fewest xGMI hops
on a single node, and data-parallel replicas are the TP groups.

The map-reduce pipeline only needs tiny DP collectives:
variable-length UTF-8 payloads (summaries, token counts) are all-gathered as
``uint8`` device tensors after an all-gather of their lengths -- one RCCL
all-gather of ``world x max_len`` bytes per phase.  TP all-reduces are issued
by the model (``engine/model.py: LlamaModel._all_reduce``: the one-shot P2P
kernel of ``parallel/custom_ar.py`` for decode-sized messages, RCCL above).

Failure discipline: a rank-local error must never make one rank skip a
collective its peers enter.  Stage-level code (``engine/provider.py``) catches
engine errors locally, still enters every collective of the stage, and turns
the error into records that the all-gather hands to EVERY rank, so retry
decisions are identical everywhere.  The process-group timeout
(``MRSUM_DIST_TIMEOUT`` seconds, default 600) bounds what cannot be caught that
way (a rank dying inside a TP all-reduce).
"""

from __future__ import annotations

import datetime
import json
import logging
import os
import sys
from dataclasses import dataclass
from typing import Any, List, Optional

import torch
import torch.distributed as dist

log = logging.getLogger("mrsum.dist")


@dataclass
class ParallelState:
    world: int = 1
    rank: int = 0
    local_rank: int = 0
    tp: int = 1
    tp_rank: int = 0
    dp: int = 1
    dp_rank: int = 0
    tp_group: Any = None
    backend: str = "none"

    @property
    def distributed(self) -> bool:
        return self.world > 1


_STATE = ParallelState()


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def init_distributed_from_env(backend: Optional[str] = None, timeout_s: Optional[float] = None) -> bool:
    """Initialise the default group when launched by torchrun (WORLD_SIZE > 1)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    force = os.environ.get("MRSUM_FORCE_DIST", "0") == "1" and "RANK" in os.environ  # world-1 RCCL rehearsal
    if (ws <= 1 and not force) or is_initialized():
        return is_initialized()
    if backend is None:
        backend = os.environ.get("MRSUM_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if timeout_s is None:
        timeout_s = float(os.environ.get("MRSUM_DIST_TIMEOUT", "600"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    kwargs = {}
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        kwargs["device_id"] = torch.device("cuda", local_rank)
    dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kwargs)
    log.info("process group up: backend=%s rank=%d/%d", backend, dist.get_rank(), dist.get_world_size())
    return True


def setup_parallel(tp: int = 1) -> ParallelState:
    """Create (or return) the DP x TP layout for ``tp`` ranks per replica."""
    global _STATE
    if not is_initialized():
        _STATE = ParallelState(tp=1, backend="none")
        if tp != 1:
            raise ValueError("tp=%d requires a process group (launch with torchrun)" % tp)
        return _STATE
    world, rank = dist.get_world_size(), dist.get_rank()
    if world % tp:
        raise ValueError("world size %d is not divisible by tp=%d" % (world, tp))
    if _STATE.world == world and _STATE.tp == tp and _STATE.backend != "none":
        return _STATE
    tp_group = None
    if tp > 1:
        for start in range(0, world, tp):
            g = dist.new_group(list(range(start, start + tp)))
            if start <= rank < start + tp:
                tp_group = g
    _STATE = ParallelState(world=world, rank=rank, local_rank=int(os.environ.get("LOCAL_RANK", rank)), tp=tp,
                           tp_rank=rank % tp, dp=world // tp, dp_rank=rank // tp, tp_group=tp_group,
                           backend=dist.get_backend())
    return _STATE


def state() -> ParallelState:
    return _STATE


_TP_GROUPS = {}


def tp_group_for(tp: int):
    """Process group of this rank's ``tp`` consecutive ranks (created once per degree; the
    whole-world degree uses the default group).  Every rank must call this with the same ``tp``."""
    if not is_initialized():
        return None
    world, rank = dist.get_world_size(), dist.get_rank()
    if world % tp:
        raise ValueError("world %d not divisible by tp %d" % (world, tp))
    if tp == world:
        return dist.group.WORLD
    if tp not in _TP_GROUPS:
        mine = None
        for start in range(0, world, tp):
            g = dist.new_group(list(range(start, start + tp)))
            if start <= rank < start + tp:
                mine = g
        _TP_GROUPS[tp] = mine
    return _TP_GROUPS[tp]


def _comm_device() -> torch.device:
    if is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_gather_bytes(payload: bytes, group=None) -> List[bytes]:
    """Gather one variable-length byte string from every rank (rank order)."""
    if not is_initialized():
        return [payload]
    dev = _comm_device()
    ws = dist.get_world_size(group)
    n = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(sizes, n, group=group)
    lens = [int(s.item()) for s in sizes]
    m = max(1, max(lens))
    buf = torch.zeros(m, dtype=torch.uint8, device=dev)
    if payload:
        buf[: len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
    outs = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(outs, buf, group=group)
    return [bytes(o[:l].cpu().numpy().tobytes()) for o, l in zip(outs, lens)]


def all_gather_json(obj: Any, group=None) -> List[Any]:
    return [json.loads(b.decode("utf-8")) for b in all_gather_bytes(json.dumps(obj).encode("utf-8"), group)]


def broadcast_json(obj: Any, src: int = 0, group=None) -> Any:
    if not is_initialized():
        return obj
    return all_gather_json(obj if dist.get_rank() == src else None, group)[src]


def barrier() -> None:
    if is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(x: float) -> float:
    if not is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_comm_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class AsyncWorks:
    """Scope of asynchronous collectives (``async_op=True`` work handles): every handle registered with
    ``add`` is waited on leaving the scope, on the normal path AND when an exception unwinds through it, so no
    work handle outlives the code that started it.  A handle left un-waited holds the backend's pending work
    until process teardown, where gloo aborts (``terminate called without an active exception``) or RCCL
    reports an unfinished collective.  Waiting on a finished work is cheap; on the exception path a wait
    error is swallowed (the original exception propagates), and a peer that never posts its side ends the
    wait at the process-group timeout.

    Only PENDING handles are kept: ``wait(work)`` waits and drops the handle at once.  A finished RCCL
    WorkNCCL still pins its output tensors while it lives, so a scope that kept every handle of a layer-major
    prefill would hold every layer's reduce-scatter / all-reduce output (and every CP K/V gather buffer)
    until the prefill ends -- O(layers x pass activations) of extra HBM."""

    def __init__(self):
        self._works = []

    def add(self, work):
        if work is not None:
            self._works.append(work)
        return work

    def wait(self, work) -> None:
        """Wait on ``work`` (a handle from ``add``, or None) and stop tracking it."""
        if work is None:
            return
        for i, w in enumerate(self._works):
            if w is work:
                del self._works[i]
                break
        work.wait()

    def __len__(self) -> int:
        return len(self._works)

    def __enter__(self) -> "AsyncWorks":
        return self

    def __exit__(self, et, ev, tb) -> bool:
        works, self._works = self._works, []
        for w in works:
            try:
                w.wait()
            except Exception:
                if et is None:
                    raise
        return False


def exit_process(code: int) -> None:
    """Leave the process with ``code`` once its work is done and the groups are torn down (``shutdown``):
    the one exit path of bench.py and the CLI (``python -m llm_map_reduce_summarizer_amd``).

    A rank of a multi-process job leaves through ``os._exit`` after flushing stdout / stderr: interpreter
    finalisation would run the C++ destructors of the communication backends, which in round 4 aborted a
    finished world-8 job once (SIGABRT after a good result; gloo's ``terminate called without an active
    exception``); the round-5 AsyncWorks scope waits every async work before its frame ends and ``shutdown``
    destroys the groups in a fixed order, after which the abort did not recur, but no destructor is left to
    chance after the result is out.  A single process that never formed a group exits normally: its atexit
    work includes a profiler's flush (rocprofv3 writes its traces there; ``os._exit`` would drop them)."""
    try:
        sys.stdout.flush()
        sys.stderr.flush()
    except Exception:  # noqa: BLE001 -- closed streams must not change the exit code
        pass
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 or os.environ.get("MRSUM_FORCE_DIST") == "1":
        logging.shutdown()
        os._exit(int(code))
    sys.exit(int(code))


def shutdown() -> None:
    """Tear the process groups down in a fixed order on every rank: a barrier (no rank leaves while a peer is
    still inside a collective), then every subgroup this module created (TP groups), then the default group.
    Each step runs even if an earlier one raised; the first error is re-raised at the end."""
    global _STATE
    if not is_initialized():
        _STATE = ParallelState()
        return
    err = None
    try:
        barrier()
    except Exception as e:  # noqa: BLE001 -- still tear down
        err = e
    subgroups = [g for g in list(_TP_GROUPS.values()) + [_STATE.tp_group]
                 if g is not None and g is not dist.group.WORLD]
    seen = set()
    for g in subgroups:
        if id(g) in seen:
            continue
        seen.add(id(g))
        try:
            dist.destroy_process_group(g)
        except Exception as e:  # noqa: BLE001
            err = err or e
    _TP_GROUPS.clear()
    _STATE = ParallelState()
    try:
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        err = err or e
    import gc
    gc.collect()
    if err is not None:
        raise err
