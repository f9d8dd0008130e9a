"""Multi-process launcher: one worker process per GPU (or per simulated CPU rank).

``spawn(fn, nprocs, args)`` starts ``nprocs`` fresh processes (``spawn`` start method, so no HIP
state is inherited), each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT set, runs ``fn(rank, *args)`` and propagates failures.  This is what
``Model.train(n_gpus=N)`` uses in place of the reference's single-process MirroredStrategy towers
(model.py:114-121).  For benchmarking, ``torch.distributed.run`` (torchrun) is equivalent.
"""
from __future__ import annotations

import os
import socket

import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _entry(rank, fn, nprocs, port, env, args):
    os.environ.update(env)
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(nprocs)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    fn(rank, *args)


def spawn(fn, nprocs, args=(), env=None, join=True):
    port = free_port()
    env = dict(env or {})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return mp.spawn(_entry, args=(fn, nprocs, port, env, args), nprocs=nprocs, join=join)
