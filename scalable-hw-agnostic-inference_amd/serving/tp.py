"""Tensor-parallel serving: one process per GPU of a TP group behind ONE HTTP front end.

The reference serves its large models sharded inside a single process that drives many
NeuronCores: vLLM ``LLM(**vllm_config)`` with ``tensor_parallel_size: 32``
(app/vllm_model_api.py:33-34,127-129; cova/mllama-32-11b-vllm-trn1-config.yaml:9), the Flux
transformer as TP8 NEFFs (app/flux_model_api.py:128-140) and T5 from ``tp_*.pt`` shards
(app/flux_model_api.py:312-314, app/t5_model_api.py:27,33).  On MI355X a TP group is N processes
(``torch.distributed.run --nproc-per-node N``, launched by the supervisor for ``WorkerSpec.tp = N``),
one per GPU, with the model's collectives on RCCL over xGMI (or the P2P all-reduce kernel).

SPMD protocol:

* every rank builds the same sharded engine (``set_device(LOCAL_RANK)`` + ``init_distributed``);
* rank 0 (the *leader*) binds the HTTP port and owns the request queue;
* before each engine call the leader broadcasts a small control message -- the method name and its
  arguments (diffusion / encoder engines: :class:`SPMDProxy`), or an LLM step with the requests
  admitted since the last step (:meth:`LLMService` with a channel) -- and the *followers*
  (:func:`follow`) execute exactly the same call, so every collective inside it lines up.

Control messages travel on a separate **gloo** group (host sockets), never on the RCCL
communicator: an idle follower blocks in a CPU receive, not in a GPU collective, and the leader sends
a heartbeat every ``HEARTBEAT_S`` seconds.

Failure handling (a TP group is one unit: it serves or it is restarted whole):

* after every CALL the leader broadcasts its outcome (ok, or the type of the exception it raised); a follower
  whose call fails stays in the group only when its exception is a mirrored input error (``MIRRORED``) AND the
  leader raised the same type -- a rank-local ``KeyError`` thrown after a collective is not excused by the
  leader's success -- and so does a follower whose call succeeded where the leader's failed with anything but a
  mirrored error.  A follower error outside ``MIRRORED`` leaves at once, without waiting for the outcome (the
  leader may be blocked in a collective the follower never joins).  Any other follower failure is reported to the
  leader on a
  second gloo group and exits non-zero; ``torch.distributed.run`` then stops the other ranks and the
  supervisor relaunches the group.  The leader's status listener marks the process broken
  (``utils.liveness.mark_broken``: ``/health`` 503) the moment the report -- or the lost connection of a
  killed follower -- arrives, so the router drains the replica before the launcher has torn it down;
* a follower that hears nothing from the leader (no call, no heartbeat) for ``LEADER_TIMEOUT_S``
  (default 2 x ``HEARTBEAT_S`` + 5 s) while idle takes the leader for dead and exits non-zero (a killed
  leader's closed socket fails the pending receive at once).
"""
from __future__ import annotations

import datetime
import os
import pickle
import threading
import time
from dataclasses import dataclass
from typing import Any, Iterable, Optional

import torch
import torch.distributed as dist

from ..utils.logging import get_logger

_log = get_logger("tp-serving")

CALL, STEP, NOOP, STOP, OUTCOME = 1, 2, 3, 4, 5
HEARTBEAT_S = float(os.environ.get("SHAI_TP_HEARTBEAT_S", "20"))
LEADER_TIMEOUT_S = float(os.environ.get("SHAI_TP_LEADER_TIMEOUT_S", str(2 * HEARTBEAT_S + 5)))
# exceptions a follower treats as mirrored on the leader (same inputs, same code -> the leader's client gets
# the error); anything else is rank-local (OOM, device fault, shard-specific shape) and breaks the group
MIRRORED = (ValueError, TypeError, KeyError)
FOLLOWER_FAILED_EXIT = 70


class TPChannel:
    """Leader -> followers control messages: an int64 header [kind, nbytes] + an optional pickled payload,
    both broadcast from rank 0 over a dedicated gloo group.  Thread-safe on the sending side."""

    def __init__(self, timeout_s: float = 3600.0):
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))
        # followers -> leader failure reports (point to point, leader receives from any rank)
        self.status_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(days=7))
        self._lock = threading.Lock()
        self.sent = 0
        self.stopping = False

    @property
    def is_leader(self) -> bool:
        return self.rank == 0

    def send(self, kind: int, payload: Any = None) -> None:
        assert self.is_leader, "only rank 0 sends control messages"
        data = pickle.dumps(payload, protocol=pickle.HIGHEST_PROTOCOL) if payload is not None else b""
        with self._lock:
            dist.broadcast(torch.tensor([kind, len(data)], dtype=torch.int64), 0, group=self.group)
            if data:
                dist.broadcast(torch.frombuffer(bytearray(data), dtype=torch.uint8), 0, group=self.group)
            self.sent += 1

    def report_failure(self, detail: str) -> None:
        """Follower: tell the leader this rank is failing (best effort; the exit that follows is what counts)."""
        data = detail.encode()[:4000]
        dist.send(torch.tensor([self.rank, len(data)], dtype=torch.int64), 0, group=self.status_group)
        if data:
            dist.send(torch.frombuffer(bytearray(data), dtype=torch.uint8), 0, group=self.status_group)

    def listen_for_failures(self, on_failure) -> threading.Thread:
        """Leader: a daemon thread that waits for a follower's failure report (or the loss of its connection,
        e.g. a killed follower) and calls ``on_failure(detail)`` once."""
        def loop():
            while True:
                hdr = torch.zeros(2, dtype=torch.int64)
                try:
                    src = dist.recv(hdr, None, group=self.status_group)
                    rank, n = (int(v) for v in hdr.tolist())
                    detail = f"rank {rank}"
                    if n:
                        buf = torch.empty(n, dtype=torch.uint8)
                        dist.recv(buf, src, group=self.status_group)
                        detail += ": " + buf.numpy().tobytes().decode(errors="replace")
                except Exception as e:  # noqa: BLE001 -- a peer's socket closed (killed rank) or teardown
                    if self.stopping:
                        return
                    if "imed out" in str(e):
                        continue
                    detail = f"lost a TP rank ({type(e).__name__}: {str(e)[:200]})"
                if not self.stopping:
                    on_failure(detail)
                return
        t = threading.Thread(target=loop, daemon=True, name="tp-status")
        t.start()
        return t

    def recv(self):
        hdr = torch.zeros(2, dtype=torch.int64)
        dist.broadcast(hdr, 0, group=self.group)
        kind, n = (int(v) for v in hdr.tolist())
        payload = None
        if n:
            buf = torch.empty(n, dtype=torch.uint8)
            dist.broadcast(buf, 0, group=self.group)
            payload = pickle.loads(buf.numpy().tobytes())   # sent by our own rank 0
        return kind, payload


class SPMDProxy:
    """Wraps an engine on the leader: calling one of ``methods`` first broadcasts (name, args, kwargs) so
    every follower runs the same call, then runs it locally.  Other attributes pass through untouched."""

    def __init__(self, target, channel: TPChannel, methods: Iterable[str]):
        self._target, self._channel, self._methods = target, channel, set(methods)

    def __getattr__(self, name):
        attr = getattr(self._target, name)
        if name not in self._methods:
            return attr

        def call(*args, **kwargs):
            from ..parallel.comm import raise_if_p2p_error
            self._channel.send(CALL, (name, args, kwargs))
            try:
                out = attr(*args, **kwargs)
                raise_if_p2p_error()
            except BaseException as e:
                # the follower compares the type NAME and requires both sides mirrored (a ValueError subclass such
                # as JSONDecodeError raised on both ranks is as mirrored as a ValueError)
                self._channel.send(OUTCOME, (type(e).__name__, isinstance(e, MIRRORED)))
                raise
            self._channel.send(OUTCOME, "")
            return out
        return call


def _die(code: int) -> None:
    """Leave NOW: a broken TP rank must not linger in a destructor or a collective that never completes."""
    import logging
    import sys
    logging.shutdown()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)


class _LeaderWatchdog:
    """Follower: exits the process when no control message (call, step or heartbeat) arrived for ``timeout_s``
    while the follower sat idle in its receive (the time a call runs does not count)."""

    def __init__(self, timeout_s: float, on_dead=None):
        self.timeout_s = timeout_s
        self.on_dead = on_dead or (lambda: _die(FOLLOWER_FAILED_EXIT))
        self.idle_since: Optional[float] = None
        self._stop = threading.Event()
        if timeout_s > 0:
            threading.Thread(target=self._loop, daemon=True, name="tp-leader-watchdog").start()

    def _loop(self):
        while not self._stop.wait(min(1.0, self.timeout_s / 4)):
            t0 = self.idle_since
            if t0 is not None and time.monotonic() - t0 > self.timeout_s:
                _log.error("leader silent: exiting", extra={"event": "leader_lost",
                                                            "detail": f"{self.timeout_s:.0f}s without a message"})
                self.on_dead()
                return

    def stop(self):
        self._stop.set()


def follow(target, channel: TPChannel, step_fn=None, leader_timeout_s: Optional[float] = None) -> int:
    """Follower main loop: execute the leader's calls until STOP.  ``step_fn(payload)`` handles STEP
    messages (the LLM engine loop).  After a CALL the follower waits for the leader's OUTCOME: a ``MIRRORED``
    (input) error that the leader raised too is logged and skipped -- the leader reports it to its client.  Any
    other divergence (a follower error the leader did not share, or a leader failure outside ``MIRRORED`` the
    follower did not share) is rank-local: it is reported to the leader and the process exits non-zero, so the
    group is restarted whole instead of running on with mismatched collectives.  Returns the number of calls."""
    n = 0
    dog = _LeaderWatchdog(LEADER_TIMEOUT_S if leader_timeout_s is None else leader_timeout_s)

    def leader_outcome():
        """("", False) when the leader's call succeeded, else (its exception type name, whether mirrored)."""
        while True:  # heartbeats may land between the call and its outcome
            dog.idle_since = time.monotonic()
            kind, payload = channel.recv()
            dog.idle_since = None
            if kind == OUTCOME:
                return tuple(payload) if payload else ("", False)
            if kind != NOOP:
                raise RuntimeError(f"TP protocol: expected the leader's call outcome, got message kind {kind}")

    try:
        while True:
            dog.idle_since = time.monotonic()
            kind, payload = channel.recv()
            dog.idle_since = None
            if kind == STOP:
                return n
            if kind in (NOOP, OUTCOME):
                continue
            err = None
            try:
                with torch.inference_mode():
                    if kind == CALL:
                        from ..parallel.comm import raise_if_p2p_error
                        name, args, kwargs = payload
                        getattr(target, name)(*args, **kwargs)
                        raise_if_p2p_error()
                    elif kind == STEP and step_fn is not None:
                        step_fn(payload)
            except Exception as e:  # noqa: BLE001 -- classified against the leader's outcome below
                err = e
            if kind != CALL or (err is not None and not isinstance(err, MIRRORED)):
                # a rank-local failure (OOM, device fault, shard-specific error) leaves AT ONCE: the leader may be
                # blocked in a collective this rank will never join, so waiting for its OUTCOME could hang the
                # group until the collective's timeout while the heartbeats keep this rank's watchdog quiet
                if err is not None:
                    _fail(channel, err)
            else:
                try:
                    lead, lead_mirrored = leader_outcome()
                except Exception as e:  # noqa: BLE001
                    _fail(channel, e)
                if err is None:
                    if lead and not lead_mirrored:
                        _fail(channel, RuntimeError(f"leader failed with {lead} where this rank succeeded"))
                else:  # a mirrored error here: excused only when the leader raised the same type, also mirrored
                    if not (lead == type(err).__name__ and lead_mirrored):
                        _fail(channel, err)
                    _log.warning("follower call failed (mirrored on the leader)",
                                 extra={"event": "follower_error", "detail": repr(err)[:300]})
            n += 1
    finally:
        dog.stop()


def _fail(channel: TPChannel, e: BaseException) -> None:
    detail = f"{type(e).__name__}: {str(e)[:500]}"
    _log.error("follower failed: leaving the TP group", extra={"event": "follower_fatal", "detail": detail})
    try:
        channel.report_failure(detail)
    except Exception:  # noqa: BLE001
        pass
    _die(FOLLOWER_FAILED_EXIT)


def heartbeat(channel: TPChannel, stop: threading.Event) -> threading.Thread:
    """Leader thread: a NOOP every HEARTBEAT_S seconds so an idle follower never hits the gloo timeout
    (sends are serialised by the channel lock, so a NOOP only ever lands between two messages)."""
    def loop():
        while not stop.wait(HEARTBEAT_S):
            try:
                channel.send(NOOP)
            except Exception:  # group torn down at shutdown
                return
    t = threading.Thread(target=loop, daemon=True, name="tp-heartbeat")
    t.start()
    return t


@dataclass
class TPContext:
    rank: int = 0
    world: int = 1
    channel: Optional[TPChannel] = None
    _hb: Optional[threading.Event] = None

    @property
    def enabled(self) -> bool:
        return self.world > 1

    @property
    def is_leader(self) -> bool:
        return self.rank == 0

    def start_heartbeat(self) -> None:
        if self.enabled and self.is_leader and self._hb is None:
            self._hb = threading.Event()
            heartbeat(self.channel, self._hb)

    def wrap(self, engine, methods: Iterable[str]):
        """Leader: an :class:`SPMDProxy` over ``engine`` (and the idle heartbeat); TP1: ``engine`` itself."""
        if not self.enabled:
            return engine
        self.start_heartbeat()
        return SPMDProxy(engine, self.channel, methods)


def env_tp_degree() -> int:
    """TP degree from the environment: ``TENSOR_PARALLEL_SIZE`` (SURVEY 2.12's vLLM compile variable), else the
    launcher's WORLD_SIZE, else 1."""
    return int(os.environ.get("TENSOR_PARALLEL_SIZE") or os.environ.get("WORLD_SIZE") or 1)


def serve(module: str, tp: int, build_engine, create_app, methods=(), step_fn=None) -> None:
    """Common ``main()`` of a TP-capable server: relaunch as ``tp`` ranks if needed, join the group, then
    rank 0 runs ``create_app(tpc)`` under uvicorn while every other rank builds the same engine
    (``build_engine()``) and follows rank 0's calls (``step_fn(engine)`` -> STEP handler, for the LLM)."""
    if relaunch_under_torchrun(tp, module):
        return
    tpc = setup(tp)
    if tpc.enabled and not tpc.is_leader:
        eng = build_engine()
        follow(eng, tpc.channel, step_fn=step_fn(eng) if step_fn is not None else None)
        return
    from .common import run
    try:
        run(create_app(tpc))
    finally:
        shutdown(tpc)


def relaunch_under_torchrun(tp: int, module: str) -> bool:
    """A TP > 1 server started as a single process (``python -m <server>``) re-runs itself as ``tp`` ranks
    under ``torch.distributed.run`` (a child process, started before this process touches the GPU) and
    exits with its status.  Returns False (nothing done) when already launched as a group or at TP1."""
    if tp <= 1 or "WORLD_SIZE" in os.environ:
        return False
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    if module == "__main__":
        module = sys.modules["__main__"].__spec__.name
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={tp}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", "-m", module]
    _log.info("relaunching as a TP group", extra={"event": "tp_relaunch", "detail": " ".join(cmd)})
    sys.exit(subprocess.call(cmd))


def setup(tensor_parallel_size: Optional[int] = None) -> TPContext:
    """Join the TP group this process was launched into (``torch.distributed.run`` env vars).  The TP degree
    is ``tensor_parallel_size`` (e.g. from /vllm_config.yaml) and must equal WORLD_SIZE -- one replica per
    launch; data parallelism is the supervisor's job (more replicas), not the launcher's."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    tp = int(tensor_parallel_size or world)
    if tp != world:
        raise ValueError(f"tensor_parallel_size={tp} but the worker was launched with WORLD_SIZE={world}: "
                         f"launch it with --nproc-per-node={tp} (supervisor WorkerSpec.tp)")
    if world == 1:
        return TPContext()
    from ..parallel.state import init_distributed
    on_cpu = os.environ.get("DEVICE", "").lower() == "cpu"
    # SHAI_TP_BACKEND=gloo on GPUs: ranks may share a GPU (tests); the model's collectives then run on the
    # xGMI/IPC P2P kernels and gloo only coordinates
    backend = "gloo" if on_cpu else (os.environ.get("SHAI_TP_BACKEND") or None)
    init_distributed(backend=backend, tp_size=tp, device=None if on_cpu else "cuda")
    ctx = TPContext(dist.get_rank(), world, TPChannel())
    if ctx.is_leader:
        from ..utils.liveness import mark_broken
        ctx.channel.listen_for_failures(lambda why: mark_broken(f"TP group broken: {why}"))
        # heartbeats from the start: a follower that is ready first must not take a leader still loading its
        # shard for dead
        ctx.start_heartbeat()
    _log.info("tp worker up", extra={"event": "tp_up", "detail": f"rank {ctx.rank}/{world}"})
    return ctx


def shutdown(ctx: TPContext) -> None:
    if ctx.enabled and ctx.is_leader and ctx.channel is not None:
        ctx.channel.stopping = True
        if ctx._hb is not None:
            ctx._hb.set()
        try:
            ctx.channel.send(STOP)
        except Exception:
            pass
