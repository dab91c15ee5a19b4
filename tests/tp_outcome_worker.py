"""Rank worker for tests/test_tp_outcome_cpu.py: a 2-rank gloo group runs SPMDProxy (rank 0) / follow (rank 1)
over a target whose methods fail in chosen ways; rank 1 prints what it survived, or exits with
FOLLOWER_FAILED_EXIT when the failure is rank-local."""
import os
import sys

import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from shai_amd.serving import tp  # noqa: E402


class Target:
    def __init__(self, rank):
        self.rank = rank

    def ok(self):
        return "ok"

    def bad_input(self):
        raise ValueError("bad prompt")            # both ranks: mirrored, the group keeps serving

    def local_keyerror(self):
        if self.rank == 1:
            raise KeyError("rank-local state")    # only the follower: must not be excused as mirrored
        return "ok"

    def leader_runtime(self):
        if self.rank == 0:
            raise RuntimeError("device fault")    # only the leader, not an input error: follower leaves
        return "ok"

    def bad_json(self):
        import json
        json.loads("{not json")                   # both ranks: a ValueError SUBCLASS, still mirrored

    def collective(self):
        import torch
        if self.rank == 1:
            raise RuntimeError("out of memory")   # follower-only, BEFORE the collective the leader enters
        t = torch.ones(1)
        dist.all_reduce(t)                        # the leader blocks here: the follower must leave at once
        return "ok"


def main():
    case = sys.argv[1]
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    ch = tp.TPChannel(timeout_s=60)
    target = Target(rank)
    if rank == 0:
        def notified(detail):
            print(f"leader notified: {detail}", flush=True)
            os._exit(0)
        ch.listen_for_failures(notified)
        proxy = tp.SPMDProxy(target, ch, {"ok", "bad_input", "local_keyerror", "leader_runtime", "bad_json",
                                          "collective"})
        seq = {"mirrored": ["ok", "bad_input", "ok"], "local": ["ok", "local_keyerror"],
               "leader": ["ok", "leader_runtime"], "subclass": ["ok", "bad_json", "ok"],
               "collective": ["ok", "collective"]}[case]
        for name in seq:
            try:
                getattr(proxy, name)()
            except Exception as e:  # noqa: BLE001
                print(f"leader {name}: {type(e).__name__}", flush=True)
        ch.send(tp.STOP)
        ch.stopping = True
        print("leader done", flush=True)
    else:
        n = tp.follow(target, ch, leader_timeout_s=0)
        print(f"follower survived {n}", flush=True)
    if case in ("mirrored", "subclass"):
        # both ranks survive: neither tears its gloo connections down while the other still uses them (the leader
        # leaving right after STOP aborted a loaded follower's exchange)
        dist.barrier()


if __name__ == "__main__":
    main()
