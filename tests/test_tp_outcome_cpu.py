"""The TP call-outcome handshake (serving/tp.py): after every mirrored CALL the leader broadcasts whether it
raised and what; a follower stays only when its own outcome matches (or the leader's was a mirrored input error)
-- the round-4 follower excused any ValueError / TypeError / KeyError, so a rank-local KeyError thrown after a
collective desynchronised the group instead of restarting it."""
import os
import socket
import subprocess
import sys

import pytest

from shai_amd.serving import tp

HERE = os.path.dirname(__file__)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(case):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), WORLD_SIZE="2",
               OMP_NUM_THREADS="1")
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "tp_outcome_worker.py"), case], env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append((p.returncode, out))
    return outs


def test_mirrored_input_error_keeps_the_group():
    (rc0, out0), (rc1, out1) = _run("mirrored")
    assert rc0 == 0 and "leader bad_input: ValueError" in out0, out0
    assert rc1 == 0 and "follower survived 3" in out1, out1


def test_rank_local_keyerror_leaves_the_group():
    (rc0, out0), (rc1, out1) = _run("local")
    assert rc1 == tp.FOLLOWER_FAILED_EXIT, out1
    assert "follower survived" not in out1
    assert "leader notified: rank 1: KeyError" in out0, out0


def test_mirrored_subclass_keeps_the_group():
    """JSONDecodeError (a ValueError subclass) raised by both ranks is mirrored: the leader sends (type name,
    isinstance(e, MIRRORED)) and the follower matches the name and the flag."""
    (rc0, out0), (rc1, out1) = _run("subclass")
    assert rc0 == 0 and "leader bad_json: JSONDecodeError" in out0, out0
    assert rc1 == 0 and "follower survived 3" in out1, out1


def test_follower_error_before_collective_leaves_at_once():
    """A follower-only RuntimeError before a collective the leader enters: the follower must report and exit
    without waiting for the leader's OUTCOME (which never comes: the leader is blocked in the all-reduce)."""
    (rc0, out0), (rc1, out1) = _run("collective")
    assert rc1 == tp.FOLLOWER_FAILED_EXIT, out1
    assert "leader notified: rank 1: RuntimeError: out of memory" in out0, out0


def test_leader_only_failure_leaves_the_group():
    (rc0, out0), (rc1, out1) = _run("leader")
    assert rc1 == tp.FOLLOWER_FAILED_EXIT, out1
    assert "leader notified: rank 1: RuntimeError: leader failed with RuntimeError" in out0, out0
